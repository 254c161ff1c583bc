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


def hip_pack_ok(compression, tensor) -> bool:
    """Compression.bf16/fp16 of a contiguous fp32 GPU tensor runs on the fused HIP pack/unpack
    kernels (cast + scale in one pass each way; csrc/kernels/optim.hip)."""
    if compression.wire_dtype not in (torch.bfloat16, torch.float16):
        return False
    if not (tensor.is_cuda and tensor.dtype == torch.float32 and tensor.is_contiguous() and tensor.numel() % 4 == 0):
        return False
    from .. import _native

    return _native.load_kernels()


def hip_pack(compression, tensor, scale: float = 1.0, out: torch.Tensor | None = None):
    """Cast (+ scale) ``tensor`` onto the 16-bit wire; ``out`` is a persistent wire buffer (e.g. the
    DistributedOptimizer's per-bucket one), so nothing is allocated per step."""
    if out is not None and out.numel() == tensor.numel() and out.dtype == compression.wire_dtype:
        wire = out
    else:
        wire = torch.empty(tensor.numel(), dtype=compression.wire_dtype, device=tensor.device)
    op = torch.ops.mihvd.scale_cast_bf16 if compression.wire_dtype == torch.bfloat16 else torch.ops.mihvd.scale_cast_f16
    op(tensor.view(-1), wire, float(scale))
    return wire


def hip_unpack(wire, out, scale: float = 1.0):
    op = torch.ops.mihvd.bf16_to_f32 if wire.dtype == torch.bfloat16 else torch.ops.mihvd.f16_to_f32
    op(wire, out.view(-1), float(scale))
    return out


class Compression:
    none = NoneCompressor
    fp16 = FP16Compressor
    bf16 = BF16Compressor
