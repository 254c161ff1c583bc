"""Collectives as ``torch.library`` custom ops: ``torch.ops.mihvd_dist.*``.

Horovod bridges framework tensors into its engine with custom framework ops (``HorovodAllreduce``
/ ``HorovodBroadcast`` / ``HorovodAllgather`` in ``horovod/tensorflow/mpi_ops.cc``) so a graph can
contain collectives with gradients. Here the same role is played by registered PyTorch operators:
they appear as single nodes to autograd, ``torch.compile``/``make_fx`` (fake/meta kernels give the
output shapes without running a collective) and ``torch.export``, and they dispatch to the mihvd
collectives (RCCL over xGMI on MI355X, gloo on CPU; negotiated when ``MIHVD_NEGOTIATE=1``).

    allreduce(Tensor t, int op=Average, str name) -> Tensor            grad: allreduce(grad, op)
    allreduce_(Tensor(a!) t, int op, str name) -> ()                   in place
    allgather(Tensor t, str name) -> Tensor                            grad: allreduce(grad) sliced to this rank
    broadcast(Tensor t, int root_rank, str name) -> Tensor             grad: grad summed onto the root
    reducescatter(Tensor t, int op, str name) -> Tensor                grad: allgather(grad)

Autograd rules follow Horovod's (``horovod/torch/mpi_ops.py`` HorovodAllreduce/Allgather/
Broadcast functions).
"""
from __future__ import annotations

import torch

from ..basics import ReduceOp

NS = "mihvd_dist"


def _coll():
    from ..parallel import collectives

    return collectives


@torch.library.custom_op(f"{NS}::allreduce", mutates_args=())
def allreduce(t: torch.Tensor, op: int = 0, name: str = "tensor") -> torch.Tensor:
    return _coll().allreduce(t, op=ReduceOp(op), name=name)


@allreduce.register_fake
def _(t, op=0, name="tensor"):
    return torch.empty_like(t)


def _allreduce_bwd(ctx, grad):
    op = ReduceOp(ctx.op)
    if op not in (ReduceOp.Average, ReduceOp.Sum):
        raise RuntimeError("mihvd_dist.allreduce: gradient defined for Average/Sum only")
    return allreduce(grad.contiguous(), int(op), ctx.name + ".grad"), None, None


def _allreduce_ctx(ctx, inputs, output):
    ctx.op = inputs[1] if len(inputs) > 1 else 0
    ctx.name = inputs[2] if len(inputs) > 2 else "tensor"


allreduce.register_autograd(_allreduce_bwd, setup_context=_allreduce_ctx)


@torch.library.custom_op(f"{NS}::allreduce_", mutates_args=("t",))
def allreduce_(t: torch.Tensor, op: int = 0, name: str = "tensor") -> None:
    _coll().allreduce_(t, op=ReduceOp(op), name=name)


@allreduce_.register_fake
def _(t, op=0, name="tensor"):
    return None


@torch.library.custom_op(f"{NS}::allgather", mutates_args=())
def allgather(t: torch.Tensor, name: str = "tensor") -> torch.Tensor:
    return _coll().allgather(t, name=name)


@allgather.register_fake
def _(t, name="tensor"):
    # dim 0 is the sum of every rank's dim 0: unknown at trace time
    n = torch.library.get_ctx().new_dynamic_size()
    return t.new_empty((n,) + tuple(t.shape[1:]))


def _allgather_ctx(ctx, inputs, output):
    ctx.dim0 = inputs[0].shape[0]
    ctx.name = inputs[1] if len(inputs) > 1 else "tensor"


def _allgather_bwd(ctx, grad):
    from .. import basics

    g = allreduce(grad.contiguous(), int(ReduceOp.Sum), ctx.name + ".grad")
    sizes = _coll().allgather_object(ctx.dim0)
    start = sum(sizes[:basics.rank()])
    return g[start:start + ctx.dim0], None


allgather.register_autograd(_allgather_bwd, setup_context=_allgather_ctx)


@torch.library.custom_op(f"{NS}::broadcast", mutates_args=())
def broadcast(t: torch.Tensor, root_rank: int, name: str = "tensor") -> torch.Tensor:
    return _coll().broadcast(t, root_rank=root_rank, name=name)


@broadcast.register_fake
def _(t, root_rank, name="tensor"):
    return torch.empty_like(t)


def _broadcast_ctx(ctx, inputs, output):
    ctx.root = inputs[1]
    ctx.name = inputs[2] if len(inputs) > 2 else "tensor"


def _broadcast_bwd(ctx, grad):
    from .. import basics

    g = allreduce(grad.contiguous(), int(ReduceOp.Sum), ctx.name + ".grad")
    return (g if basics.rank() == ctx.root else torch.zeros_like(g)), None, None


broadcast.register_autograd(_broadcast_bwd, setup_context=_broadcast_ctx)


@torch.library.custom_op(f"{NS}::reducescatter", mutates_args=())
def reducescatter(t: torch.Tensor, op: int = 0, name: str = "tensor") -> torch.Tensor:
    return _coll().reducescatter(t, op=ReduceOp(op), name=name)


@reducescatter.register_fake
def _(t, op=0, name="tensor"):
    n = torch.library.get_ctx().new_dynamic_size()
    return t.new_empty((n,) + tuple(t.shape[1:]))


def _reducescatter_ctx(ctx, inputs, output):
    ctx.op = inputs[1] if len(inputs) > 1 else 0
    ctx.name = inputs[2] if len(inputs) > 2 else "tensor"


def _reducescatter_bwd(ctx, grad):
    from .. import basics

    g = allgather(grad.contiguous(), ctx.name + ".grad")
    if ReduceOp(ctx.op) == ReduceOp.Average:
        g = g / basics.size()
    return g, None, None


reducescatter.register_autograd(_reducescatter_bwd, setup_context=_reducescatter_ctx)

__all__ = ["allreduce", "allreduce_", "allgather", "broadcast", "reducescatter", "NS"]
