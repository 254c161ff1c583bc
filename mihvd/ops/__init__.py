"""Hand-written CDNA4 (gfx950) HIP kernels of the MNIST hot path, registered as ``torch.ops.mihvd``.

``load()`` loads ``mihvd/_native/libmihvd_kernels.so`` (built in-tree by ``python -m mihvd._build``)
and raises if it is unavailable. Kernels: conv1_fwd, conv2_fwd, fc1_fwd, head_fwd_bwd, fc1_wgrad,
fc1_dgrad, conv2_bwd (+ fused conv1 wgrad), conv2_wgrad_reduce, adam_step, scale_cast_bf16, bf16_to_f32,
segment_dots, adasum_combine, grad_check_, update_scale_ (csrc/kernels/*.hip).
"""
from .. import _native


def load():
    _native.require_kernels()
    import torch

    return torch.ops.mihvd


def available() -> bool:
    return _native.load_kernels()
