"""fp32 factor gather of dense/kernel's gradient rows (the fp32 data plane of SURVEY.md §5.8 / N4).

dW3 = a2^T dz has rank B per rank (a2: [B][3136] fc1 input, dz: [B][1024] fc1 output gradient), so
the reference's per-step allreduce of the 12.8 MB dense/kernel gradient
(horovod/tensorflow_mnist.py:133, hvd.DistributedOptimizer) can be replaced, when the optimizer of
W3 is sharded by rows (rank r owns rows [r R, (r + 1) R), R = 3136 / N), by moving the factors:

* all-gather of every rank's fp32 dz ([N][B][1024]), and
* all-to-all of the a2 columns of each rank's rows (rank j receives a2[:, j R:(j + 1) R] from every
  rank: [N][B][R]),

after which rank r forms its rows of the summed gradient exactly, over all N B samples, as one fp32
GEMM (R x N B x 1024). Per rank (N - 1) B (1024 + R) floats arrive instead of the reduce-scatter's
(N - 1) R 1024 (N = 8, B = 100: 3.9 MB instead of 11.2 MB).

For small N the replicated form needs no sharding at all: every rank all-gathers every rank's a2
and dz ((N - 1) B (3136 + 1024) floats, 1.66 MB per peer at B = 100, on every link at once) and forms
ALL of dW3 (factor_full_), so neither the 12.8 MB gradient nor the updated rows cross the links.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def factor_exchange_(a2: torch.Tensor, dz: torch.Tensor, dz_all: torch.Tensor, a2_send: torch.Tensor,
                     a2_recv: torch.Tensor, rank: int, world: int, comm=None):
    """The factor exchange alone: dz_all <- every rank's dz (all-gather of ``dz``, which must not
    alias ``dz_all``: a reader of ``dz`` may run beside the exchange), a2_recv[j] <- rank j's a2 columns of this rank's rows (all-to-all of [world][B][R]).
    ``comm``: a :class:`mihvd.parallel.rccl.NativeComm` (the collectives then run on the current HIP
    stream), else the default process group (nccl, or host collectives such as gloo). Collective."""
    N = world
    B = a2.shape[0]
    R = a2.shape[1] // N
    a2_send.copy_(a2.view(B, N, R).transpose(0, 1))
    if comm is not None:
        comm.all_to_all(a2_recv, a2_send)
        comm.all_gather_into(dz_all, dz)
    elif N == 1:
        a2_recv.copy_(a2_send)
        dz_all[0].copy_(dz)
    elif dist.get_backend() == "nccl":
        dist.all_to_all_single(a2_recv, a2_send)
        dist.all_gather_into_tensor(dz_all, dz)
    else:  # host collectives (gloo): the a2 blocks out of an all-gather of every rank's send buffer
        sends = [torch.empty_like(a2_send) for _ in range(N)]
        dist.all_gather(sends, a2_send)
        for j in range(N):
            a2_recv[j].copy_(sends[j][rank])
        dist.all_gather(list(dz_all.unbind(0)), dz.clone())


def factor_rows_(out: torch.Tensor, a2: torch.Tensor, dz: torch.Tensor, dz_all: torch.Tensor,
                 a2_send: torch.Tensor, a2_recv: torch.Tensor, rank: int, world: int, comm=None) -> torch.Tensor:
    """out[R][1024] = rows [rank R, (rank + 1) R) of sum over ranks of a2_q^T dz_q: the exchange, then
    one torch GEMM. The host-side reference of the exchange (tests); the trainer forms its rows with
    the hand-written ``csrc/kernels/f32_factor.hip``, which also applies Adam to them from the
    accumulators. Collective: every rank calls it."""
    factor_exchange_(a2, dz, dz_all, a2_send, a2_recv, rank, world, comm)
    N, B = world, a2.shape[0]
    R = a2.shape[1] // N
    return torch.mm(a2_recv.view(N * B, R).t(), dz_all.view(N * B, dz_all.shape[-1]), out=out)


def factor_gather_all_(a2_all: torch.Tensor, dz_all: torch.Tensor, rank: int, world: int, comm=None):
    """The replicated factor plane's exchange, in place: a2_all[q] / dz_all[q] ([N][B][3136] /
    [N][B][1024]) <- rank q's a2 / dz, this rank's slices already holding its own. ``comm``: a
    :class:`mihvd.parallel.rccl.NativeComm` (one RCCL group on the current HIP stream), else the
    default process group. Collective."""
    outs, mine = (a2_all, dz_all), (a2_all[rank], dz_all[rank])
    if comm is not None:
        comm.all_gather_many_into(outs, mine)
    elif world == 1:
        return
    elif dist.get_backend() == "nccl":
        for o, m in zip(outs, mine):
            dist.all_gather_into_tensor(o, m)
    else:  # host collectives (gloo)
        for o, m in zip(outs, mine):
            dist.all_gather(list(o.unbind(0)), m.clone())


def factor_full_(out: torch.Tensor, a2_all: torch.Tensor, dz_all: torch.Tensor, rank: int, world: int,
                 comm=None) -> torch.Tensor:
    """out[3136][1024] = sum over ranks of a2_q^T dz_q, every row on every rank (the replicated
    plane): the in-place exchange, then one torch GEMM over the N B gathered samples. The host-side
    reference; the trainer forms the rows with ``csrc/kernels/f32_factor.hip::f32_factor_full``,
    which also applies Adam to them. Collective."""
    factor_gather_all_(a2_all, dz_all, rank, world, comm)
    N, B = a2_all.shape[0], a2_all.shape[1]
    return torch.mm(a2_all.view(N * B, -1).t(), dz_all.view(N * B, -1), out=out)


__all__ = ["factor_exchange_", "factor_rows_", "factor_gather_all_", "factor_full_"]
