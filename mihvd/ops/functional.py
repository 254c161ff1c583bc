"""Autograd-facing wrappers of the CDNA4 kernels (``torch.ops.mihvd.*``) for the MNIST CNN.

* ``mnist_logits(model, images)`` — inference forward through the HIP kernels (conv1 + conv2 in one
  launch with fused bias/ReLU/pool, fc1 split-K MFMA) and a small torch epilogue for fc2.
* ``fused_mnist_loss(model, images, labels)`` — the whole forward+backward in HIP kernels,
  exposed as one autograd node: it returns the mean softmax cross-entropy and, on ``backward()``,
  hands the kernel-computed parameter gradients to autograd. This is how a stock optimizer loop
  (e.g. ``hvd.DistributedOptimizer`` with its per-parameter hooks) drives the HIP path; the fully
  fused graph-replayed loop lives in ``mihvd.models.fused_mnist``.

Both take ``precision``: ``"bf16"`` (bf16 MFMA operands, fp32 accumulation; the default),
``"fp16"`` (the same kernels compiled with IEEE fp16 operands, v_mfma_f32_16x16x32_f16 — the
Keras ``mixed_float16`` policy; its backward runs loss-scaled, see ``fused_mnist_loss``) or
``"fp32"`` (the exact-fp32 kernels of csrc/kernels/f32_*.hip); ``MNISTConvNet.hip_precision``
sets it for the model's own forward.
"""
from __future__ import annotations

import os

import torch

from .. import _native
from ..models.mnist import FC1_KS, TF_PARAM_ORDER


class _Workspace:
    """Per-(device, batch) activation/gradient buffers reused across calls."""

    _cache: dict = {}

    @classmethod
    def get(cls, device, B, dtype=torch.bfloat16):
        key = (str(device), B, dtype)
        ws = cls._cache.get(key)
        if ws is None:
            ops = torch.ops.mihvd
            f32 = dict(device=device, dtype=torch.float32)
            bf = dict(device=device, dtype=dtype)  # the 16-bit operand format (bf16 or fp16)
            u8 = dict(device=device, dtype=torch.uint8)
            ws = dict(
                a1=torch.empty(B, 14, 14, 32, **bf), idx1=torch.empty(B, 14, 14, 32, **u8),
                a2=torch.empty(B, 3136, **bf), idx2=torch.empty(B, 3136, **u8), zpart=torch.empty(FC1_KS, B, 1024, **f32),
                h=torch.empty(B, 1024, **bf), dz=torch.empty(B, 1024, **bf), dlog=torch.empty(B, 10, **f32),
                stats=torch.empty(B, 2, **f32), g2=torch.empty(B, 3136, **bf),
                cpart=torch.empty(B, 896, **f32), slab=torch.empty(int(ops.conv2_wgrad_groups(B)), 51200, **f32),
                state=torch.zeros(4, device=device, dtype=torch.int64),
                w1bf=torch.empty(800, **bf), w2bf=torch.empty(51200, **bf), w3bf=torch.empty(3136 * 1024, **bf),
            )
            cls._cache[key] = ws
        return ws


class _WorkspaceF32:
    """Per-(device, batch) buffers of the exact-fp32 kernels."""

    _cache: dict = {}

    @classmethod
    def get(cls, device, B):
        key = (str(device), B)
        ws = cls._cache.get(key)
        if ws is None:
            ops = torch.ops.mihvd
            f32 = dict(device=device, dtype=torch.float32)
            u8 = dict(device=device, dtype=torch.uint8)
            ws = dict(
                a1=torch.empty(B, 14, 14, 32, **f32), idx1=torch.empty(B, 14, 14, 32, **u8),
                a2=torch.empty(B, 3136, **f32), idx2=torch.empty(B, 3136, **u8), zpart=torch.empty(14, B, 1024, **f32),
                h=torch.empty(B, 1024, **f32), dz=torch.empty(B, 1024, **f32), dlog=torch.empty(B, 10, **f32),
                stats=torch.empty(B, 2, **f32), dY2=torch.empty(B, 14, 14, 64, **f32),
                db2p=torch.empty(int(ops.f32_db2_rows(B)), 64, **f32),
                slab=torch.empty(int(ops.f32_wgrad_groups(B)), 51200, **f32),
                cpart=torch.empty(int(ops.f32_dgrad_blocks(B)), 832, **f32),
                state=torch.zeros(4, device=device, dtype=torch.int64),
            )
            cls._cache[key] = ws
        return ws


class _Ops16:
    """The 16-bit-operand kernel set: torch.ops.mihvd.<op> (bf16) or <op>_f16 (the fp16 build)."""

    def __init__(self, fp16: bool):
        o = torch.ops.mihvd
        sfx = "_f16" if fp16 else ""
        self.dtype = torch.float16 if fp16 else torch.bfloat16
        self.cast = o.scale_cast_f16 if fp16 else o.scale_cast_bf16
        for n in ("conv1_fwd", "conv2_fwd", "conv12_fwd", "fc1_fwd", "head_fwd_bwd", "fc1_bwd", "conv2_bwd"):
            setattr(self, n, getattr(o, n + sfx))
        self.conv2_wgrad_reduce = o.conv2_wgrad_reduce  # fp32 partials: format-free


def _ops16(precision):
    return _Ops16(precision == "fp16")


def _conv_forward(ops, ws, x, st, w1, b1, b2):
    """conv1 + conv2 forward: one conv12 launch (conv1 on MFMA, 16-bit operands, like the fused
    trainer) unless MIHVD_CONV12=0 (conv1 as an fp32 VALU convolution, then conv2)."""
    if os.environ.get("MIHVD_CONV12", "1") != "0":
        ops.cast(w1.reshape(-1), ws["w1bf"], 1.0)
        ops.conv12_fwd(x, None, st, ws["w1bf"], b1, ws["w2bf"], b2, ws["a1"], ws["idx1"], ws["a2"], ws["idx2"])
        return
    ops.conv1_fwd(x, None, st, w1.reshape(-1), b1, ws["a1"], ws["idx1"])
    ops.conv2_fwd(ws["a1"], ws["w2bf"], b2, ws["a2"], ws["idx2"])


def _params(model):
    named = dict(model.ordered_parameters())
    return [named[n] for n in TF_PARAM_ORDER]


@torch.no_grad()
def mnist_logits(model, images: torch.Tensor, precision: str | None = None) -> torch.Tensor:
    _native.require_kernels()
    ops = torch.ops.mihvd
    x = images.reshape(-1, 784).float().contiguous()
    B = x.shape[0]
    precision = precision or getattr(model, "hip_precision", "bf16")
    if B > 128:
        return torch.cat([mnist_logits(model, x[i:i + 128], precision) for i in range(0, B, 128)])
    w1, b1, w2, b2, w3, b3, w4, b4 = _params(model)
    if precision == "fp32":
        ws = _WorkspaceF32.get(x.device, B)
        ops.f32_conv1_fwd(x, None, None, w1.detach().reshape(-1), b1.detach(), ws["a1"], ws["idx1"])
        ops.f32_conv2_fwd(ws["a1"], w2.detach(), b2.detach(), ws["a2"], ws["idx2"])
        ops.f32_fc1_fwd(ws["a2"], w3.detach(), ws["zpart"])
        h = torch.relu(ws["zpart"].sum(0) + b3)
        return h @ w4 + b4
    ops = _ops16(precision)
    ws = _Workspace.get(x.device, B, ops.dtype)
    ops.cast(w2.detach().reshape(-1), ws["w2bf"], 1.0)
    ops.cast(w3.detach().reshape(-1), ws["w3bf"], 1.0)
    _conv_forward(ops, ws, x, None, w1.detach(), b1.detach(), b2.detach())
    ops.fc1_fwd(ws["a2"], ws["w3bf"], ws["zpart"])
    h = torch.relu(ws["zpart"].sum(0) + b3)
    return (h.to(ops.dtype).float() @ w4 + b4).float()


class _FusedMNISTLossF32(torch.autograd.Function):
    """The exact-fp32 step's kernels (csrc/kernels/f32_fwd.hip, f32_bwd.hip) as one autograd node."""

    @staticmethod
    def forward(ctx, x, labels, dropout, seed, w1, b1, w2, b2, w3, b3, w4, b4):
        ops = torch.ops.mihvd
        B = x.shape[0]
        ws = _WorkspaceF32.get(x.device, B)
        grads = [torch.empty_like(p, dtype=torch.float32) for p in (w1, b1, w2, b2, w3, b3, w4, b4)]
        gW1, gb1, gW2, gb2, gW3, gb3, gW4, gb4 = grads
        st = ws["state"]
        w2c, w3c = w2.contiguous(), w3.contiguous()
        ops.f32_conv1_fwd(x, None, st, w1.reshape(-1), b1, ws["a1"], ws["idx1"])
        ops.f32_conv2_fwd(ws["a1"], w2c, b2, ws["a2"], ws["idx2"])
        ops.f32_fc1_fwd(ws["a2"], w3c, ws["zpart"])
        ops.f32_head_fwd_bwd(ws["zpart"], b3, w4.contiguous(), b4, labels, None, st, int(seed), float(dropout), ws["h"],
                             ws["dz"], ws["dlog"], ws["stats"])
        ops.f32_fc1_bwd(ws["dz"], ws["a2"], ws["idx2"], ws["h"], ws["dlog"], w3c, ws["dY2"], ws["db2p"], gW3, gb3, gW4,
                        gb4)
        ops.f32_conv2_bwd(ws["dY2"], w2c, ws["a1"], ws["idx1"], x, None, st, ws["cpart"], ws["slab"])
        ops.f32_conv_reduce(ws["slab"], ws["cpart"], ws["db2p"], gW2.reshape(-1), gW1.reshape(-1), gb1, gb2)
        st[0] += 1  # next call draws a fresh dropout mask
        ctx.save_for_backward(*grads)
        acc = ws["stats"][:, 1].mean()
        ctx.mark_non_differentiable(acc)
        return ws["stats"][:, 0].mean(), acc

    @staticmethod
    def backward(ctx, gout, _gacc):
        grads = [g * gout for g in ctx.saved_tensors]
        return (None, None, None, None, *grads)


class _FusedMNISTLoss(torch.autograd.Function):
    """The 16-bit-operand step (bf16, or fp16 with a loss-scaled backward) as one autograd node.

    ``dz_scale`` (fp16): the head writes dz = S * dL/dz (fp16 has 8 fewer exponent bits than bf16;
    dz ~ 1e-4 sits in fp16's subnormal range unscaled), so every gradient the kernels derive from
    dz — W1, b1, W2, b2, W3, b3 — comes out S-scaled (inf/NaN if a 16-bit intermediate overflowed);
    dW4 / db4 come from the fp32 dlog and are not. ``backward`` divides the former by S, so the
    node returns true gradients times the incoming ``gout`` — under a loss scaler ``gout`` is S
    and the non-finite check of the scaler sees any overflow."""

    @staticmethod
    def forward(ctx, x, labels, dropout, seed, precision, dz_scale, w1, b1, w2, b2, w3, b3, w4, b4):
        ops = _ops16(precision)
        B = x.shape[0]
        ws = _Workspace.get(x.device, B, ops.dtype)
        grads = [torch.empty_like(p, dtype=torch.float32) for p in (w1, b1, w2, b2, w3, b3, w4, b4)]
        gW1, gb1, gW2, gb2, gW3, gb3, gW4, gb4 = grads
        ops.cast(w2.reshape(-1), ws["w2bf"], 1.0)
        ops.cast(w3.reshape(-1), ws["w3bf"], 1.0)
        st = ws["state"]
        _conv_forward(ops, ws, x, st, w1, b1, b2)
        ops.fc1_fwd(ws["a2"], ws["w3bf"], ws["zpart"])
        ops.head_fwd_bwd(ws["zpart"], b3, w4, b4, labels, None, st, int(seed), float(dropout), ws["h"], ws["dz"],
                         ws["dlog"], ws["stats"], -1, float(dz_scale))
        ops.fc1_bwd(ws["dz"], ws["a2"], ws["h"], ws["dlog"], ws["w3bf"], gW3, gb3, gW4, gb4, ws["g2"])
        ops.conv2_bwd(ws["g2"], ws["idx2"], ws["a1"], ws["w2bf"], x, None, st, ws["idx1"], ws["slab"], ws["cpart"])
        ops.conv2_wgrad_reduce(ws["slab"], ws["cpart"], B, gW2.reshape(-1), gW1.reshape(-1), gb1, gb2)
        st[0] += 1  # next call draws a fresh dropout mask
        ctx.dz_scale = float(dz_scale)
        ctx.save_for_backward(*grads)
        acc = ws["stats"][:, 1].mean()
        ctx.mark_non_differentiable(acc)
        return ws["stats"][:, 0].mean(), acc

    @staticmethod
    def backward(ctx, gout, _gacc):
        inv = 1.0 / ctx.dz_scale
        grads = [g * (gout * inv) if i < 6 else g * gout for i, g in enumerate(ctx.saved_tensors)]
        return (None, None, None, None, None, None, *grads)


def fused_mnist_loss(model, images: torch.Tensor, labels: torch.Tensor, training: bool = True, seed: int = 17,
                     return_accuracy: bool = False, precision: str | None = None, loss_scale: float | None = None):
    """Mean softmax cross-entropy of the reference CNN, forward and backward in HIP kernels.

    ``loss_scale`` (``precision="fp16"``): the factor S the kernels scale dz by, normally the
    current scale of the dynamic loss scaler (default 2**15, Keras' initial scale). The returned
    gradients are the true ones times the incoming gradient either way."""
    _native.require_kernels()
    x = images.reshape(-1, 784).float().contiguous()
    if x.shape[0] > 128:
        raise ValueError("fused_mnist_loss: per-call batch must be <= 128")
    rate = model.dropout_rate if training else 0.0
    precision = precision or getattr(model, "hip_precision", "bf16")
    if precision not in ("fp32", "bf16", "fp16"):
        raise ValueError("fused_mnist_loss: precision must be fp32, bf16 or fp16 (got %r)" % (precision,))
    y = labels.long().contiguous()
    if precision == "fp32":
        loss, acc = _FusedMNISTLossF32.apply(x, y, rate, seed, *_params(model))
    else:
        S = float(loss_scale) if (precision == "fp16" and loss_scale is not None) else (
            2.0 ** 15 if precision == "fp16" else 1.0)
        loss, acc = _FusedMNISTLoss.apply(x, y, rate, seed, precision, S, *_params(model))
    return (loss, acc) if return_accuracy else loss
