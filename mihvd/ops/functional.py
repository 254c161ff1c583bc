"""Autograd-facing wrappers of the CDNA4 kernels (``torch.ops.mihvd.*``) for the MNIST CNN.

* ``mnist_logits(model, images)`` — inference forward through the HIP kernels (conv1 + conv2 in one
  launch with fused bias/ReLU/pool, fc1 split-K MFMA) and a small torch epilogue for fc2.
* ``fused_mnist_loss(model, images, labels)`` — the whole forward+backward in HIP kernels,
  exposed as one autograd node: it returns the mean softmax cross-entropy and, on ``backward()``,
  hands the kernel-computed parameter gradients to autograd. This is how a stock optimizer loop
  (e.g. ``hvd.DistributedOptimizer`` with its per-parameter hooks) drives the HIP path; the fully
  fused graph-replayed loop lives in ``mihvd.models.fused_mnist``.
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
    def get(cls, device, B):
        key = (str(device), B)
        ws = cls._cache.get(key)
        if ws is None:
            ops = torch.ops.mihvd
            f32 = dict(device=device, dtype=torch.float32)
            bf = dict(device=device, dtype=torch.bfloat16)
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


def _conv_forward(ops, ws, x, st, w1, b1, b2):
    """conv1 + conv2 forward: one conv12 launch (conv1 on MFMA, bf16 operands, like the fused
    trainer) unless MIHVD_CONV12=0 (conv1 as an fp32 VALU convolution, then conv2)."""
    if os.environ.get("MIHVD_CONV12", "1") != "0":
        ops.scale_cast_bf16(w1.reshape(-1), ws["w1bf"], 1.0)
        ops.conv12_fwd(x, None, st, ws["w1bf"], b1, ws["w2bf"], b2, ws["a1"], ws["idx1"], ws["a2"], ws["idx2"])
        return
    ops.conv1_fwd(x, None, st, w1.reshape(-1), b1, ws["a1"], ws["idx1"])
    ops.conv2_fwd(ws["a1"], ws["w2bf"], b2, ws["a2"], ws["idx2"])


def _params(model):
    named = dict(model.ordered_parameters())
    return [named[n] for n in TF_PARAM_ORDER]


@torch.no_grad()
def mnist_logits(model, images: torch.Tensor) -> torch.Tensor:
    _native.require_kernels()
    ops = torch.ops.mihvd
    x = images.reshape(-1, 784).float().contiguous()
    B = x.shape[0]
    if B > 128:
        return torch.cat([mnist_logits(model, x[i:i + 128]) for i in range(0, B, 128)])
    w1, b1, w2, b2, w3, b3, w4, b4 = _params(model)
    ws = _Workspace.get(x.device, B)
    ops.scale_cast_bf16(w2.detach().reshape(-1), ws["w2bf"], 1.0)
    ops.scale_cast_bf16(w3.detach().reshape(-1), ws["w3bf"], 1.0)
    _conv_forward(ops, ws, x, None, w1.detach(), b1.detach(), b2.detach())
    ops.fc1_fwd(ws["a2"], ws["w3bf"], ws["zpart"])
    h = torch.relu(ws["zpart"].sum(0) + b3)
    return (h.to(torch.bfloat16).float() @ w4 + b4).float()


class _FusedMNISTLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, labels, dropout, seed, w1, b1, w2, b2, w3, b3, w4, b4):
        ops = torch.ops.mihvd
        B = x.shape[0]
        ws = _Workspace.get(x.device, B)
        grads = [torch.empty_like(p, dtype=torch.float32) for p in (w1, b1, w2, b2, w3, b3, w4, b4)]
        gW1, gb1, gW2, gb2, gW3, gb3, gW4, gb4 = grads
        ops.scale_cast_bf16(w2.reshape(-1), ws["w2bf"], 1.0)
        ops.scale_cast_bf16(w3.reshape(-1), ws["w3bf"], 1.0)
        st = ws["state"]
        _conv_forward(ops, ws, x, st, w1, b1, b2)
        ops.fc1_fwd(ws["a2"], ws["w3bf"], ws["zpart"])
        ops.head_fwd_bwd(ws["zpart"], b3, w4, b4, labels, None, st, int(seed), float(dropout), ws["h"], ws["dz"],
                         ws["dlog"], ws["stats"])
        ops.fc1_bwd(ws["dz"], ws["a2"], ws["h"], ws["dlog"], ws["w3bf"], gW3, gb3, gW4, gb4, ws["g2"])
        ops.conv2_bwd(ws["g2"], ws["idx2"], ws["a1"], ws["w2bf"], x, None, st, ws["idx1"], ws["slab"], ws["cpart"])
        ops.conv2_wgrad_reduce(ws["slab"], ws["cpart"], B, gW2.reshape(-1), gW1.reshape(-1), gb1, gb2)
        st[0] += 1  # next call draws a fresh dropout mask
        ctx.save_for_backward(*grads)
        acc = ws["stats"][:, 1].mean()
        ctx.mark_non_differentiable(acc)
        return ws["stats"][:, 0].mean(), acc

    @staticmethod
    def backward(ctx, gout, _gacc):
        grads = [g * gout for g in ctx.saved_tensors]
        return (None, None, None, None, *grads)


def fused_mnist_loss(model, images: torch.Tensor, labels: torch.Tensor, training: bool = True, seed: int = 17,
                     return_accuracy: bool = False):
    """Mean softmax cross-entropy of the reference CNN, forward and backward in HIP kernels."""
    _native.require_kernels()
    x = images.reshape(-1, 784).float().contiguous()
    if x.shape[0] > 128:
        raise ValueError("fused_mnist_loss: per-call batch must be <= 128")
    rate = model.dropout_rate if training else 0.0
    loss, acc = _FusedMNISTLoss.apply(x, labels.long().contiguous(), rate, seed, *_params(model))
    return (loss, acc) if return_accuracy else loss
