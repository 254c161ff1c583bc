"""Gradient compression for the allreduce data plane (Horovod ``hvd.Compression``).

``Compression.bf16`` is the MI355X-native choice: RCCL reduces ``bfloat16`` natively over xGMI, so
the bucket is cast once, reduced at half the bytes, and cast back. ``fp16`` is kept for Horovod
parity. Casting happens on the bucket (fusion buffer), not per tensor.
"""
from __future__ import annotations

import torch


class Compressor:
    wire_dtype: torch.dtype | None = None

    @classmethod
    def compress(cls, tensor: torch.Tensor):
        return tensor, None

    @classmethod
    def decompress(cls, tensor: torch.Tensor, ctx):
        return tensor


class NoneCompressor(Compressor):
    pass


class _CastCompressor(Compressor):
    @classmethod
    def compress(cls, tensor):
        if tensor.is_floating_point() and tensor.dtype != cls.wire_dtype:
            return tensor.to(cls.wire_dtype), tensor.dtype
        return tensor, None

    @classmethod
    def decompress(cls, tensor, ctx):
        return tensor if ctx is None else tensor.to(ctx)


class FP16Compressor(_CastCompressor):
    wire_dtype = torch.float16


class BF16Compressor(_CastCompressor):
    wire_dtype = torch.bfloat16


class Compression:
    none = NoneCompressor
    fp16 = FP16Compressor
    bf16 = BF16Compressor
