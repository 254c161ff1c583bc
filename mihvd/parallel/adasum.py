"""Adasum reduction (``hvd.Adasum``; reference: ``--use-adasum``, horovod/tensorflow_mnist.py:31-32,126-127,133).

Adasum combines two gradients scale-invariantly, per tensor (layer)::

    adasum(a, b) = (1 - a.b / (2|a|^2)) a + (1 - a.b / (2|b|^2)) b

and reduces N ranks by recursive distance doubling over point-to-point exchanges (on MI355X each
exchange is a direct xGMI peer transfer via RCCL send/recv). Non-power-of-two worlds first fold the
extra ranks into their partners and send the result back at the end.

Semantics follow Horovod's GPU build: with the RCCL data plane and more than one
node, gradients are *averaged* inside the node and Adasum runs across nodes — which is why the
reference scales the learning rate by ``local_size`` when ``nccl_built()``. On a single node that
is a plain average. ``MIHVD_ADASUM_FLAT=1`` (or the gloo backend) selects flat all-rank Adasum.
The per-segment dot/norm reductions are vectorised torch ops on the bucket; on the fused MNIST path
they run in the native allreduce stage (see mihvd/models/fused_mnist.py).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.distributed as dist


def _segment_dots(a: torch.Tensor, b: torch.Tensor, segments: Sequence[tuple[int, int]]):
    """Per-segment (a.b, |a|^2, |b|^2) in float64 for stability, as three 1-D tensors."""
    a64 = a.double()
    b64 = b.double()
    if len(segments) == 1 and segments[0] == (0, a.numel()):
        return (torch.dot(a64, b64).view(1), torch.dot(a64, a64).view(1), torch.dot(b64, b64).view(1))
    ids = torch.empty(a.numel(), dtype=torch.long, device=a.device)
    ids.fill_(len(segments))  # padding goes to a dummy segment
    for i, (s, e) in enumerate(segments):
        ids[s:e] = i
    n = len(segments) + 1
    ab = torch.zeros(n, dtype=torch.float64, device=a.device).index_add_(0, ids, a64 * b64)
    aa = torch.zeros(n, dtype=torch.float64, device=a.device).index_add_(0, ids, a64 * a64)
    bb = torch.zeros(n, dtype=torch.float64, device=a.device).index_add_(0, ids, b64 * b64)
    return ab[:-1], aa[:-1], bb[:-1]


_OFFS_CACHE: dict = {}


def _covering_offsets(segments: Sequence[tuple[int, int]], n: int) -> tuple[list[int], list[int]]:
    """(offsets, plain_sum_flags) of a segment table covering [0, n): gaps between the given
    segments become segments of their own that are summed, not Adasum-combined (as in
    ``adasum_pair``'s torch path)."""
    offs, flags = [0], []
    for s, e in sorted(segments):
        if s > offs[-1]:
            offs.append(s)
            flags.append(1)
        if e > offs[-1]:
            offs.append(e)
            flags.append(0)
    if offs[-1] < n:
        offs.append(n)
        flags.append(1)
    return offs, flags


def _hip_pair(a: torch.Tensor, b: torch.Tensor, segments) -> torch.Tensor:
    """The CDNA4 path (csrc/kernels/dp_kernels.hip): one fp64-accumulated dot/norm launch and one
    streaming combine launch for all segments."""
    key = (tuple(segments), a.numel(), a.device)
    hit = _OFFS_CACHE.get(key)
    if hit is None:
        offs, flags = _covering_offsets(segments, a.numel())
        max_len = max(e - s for s, e in zip(offs[:-1], offs[1:]))
        hit = (torch.tensor(offs + flags, dtype=torch.int64, device=a.device), max_len,
               torch.empty(3 * (len(offs) - 1), dtype=torch.float64, device=a.device))
        _OFFS_CACHE[key] = hit
    offs_dev, max_len, dots = hit
    ops = torch.ops.mihvd
    a, b = a.contiguous(), b.contiguous()
    ops.segment_dots(a, b, offs_dev, max_len, dots)
    out = torch.empty_like(a)
    ops.adasum_combine(a, b, offs_dev, max_len, dots, out)
    return out


def _use_hip(a: torch.Tensor) -> bool:
    if not (a.is_cuda and a.dtype == torch.float32):
        return False
    from .. import _native

    _native.require_kernels()  # a GPU tensor must take the HIP path: fail loudly if it is missing
    return True


def adasum_pair(a: torch.Tensor, b: torch.Tensor, segments: Sequence[tuple[int, int]] | None = None) -> torch.Tensor:
    """Combine two flat vectors segment by segment. ``a`` must be the lower-rank operand so both
    partners compute bit-identical results. fp32 GPU vectors run the HIP kernels; everything else
    (CPU/gloo, other dtypes) the torch formulation below, which is also the test oracle."""
    if segments is None:
        segments = [(0, a.numel())]
    if _use_hip(a):
        return _hip_pair(a, b, segments)
    ab, aa, bb = _segment_dots(a, b, segments)
    ca = torch.where(aa > 0, 1.0 - ab / (2.0 * aa), torch.zeros_like(aa))
    cb = torch.where(bb > 0, 1.0 - ab / (2.0 * bb), torch.zeros_like(bb))
    # |a| == 0 -> result is b (cb = 1 - 0 = 1); |b| == 0 -> result is a.
    ca = torch.where(bb > 0, ca, torch.ones_like(ca))
    cb = torch.where(aa > 0, cb, torch.ones_like(cb))
    out = torch.empty_like(a)
    covered = 0
    for i, (s, e) in enumerate(segments):
        out[s:e] = a[s:e] * ca[i].to(a.dtype) + b[s:e] * cb[i].to(a.dtype)
        covered += e - s
    if covered != a.numel():  # padding between segments: plain sum (it is zero anyway)
        mask = torch.ones(a.numel(), dtype=torch.bool, device=a.device)
        for s, e in segments:
            mask[s:e] = False
        out[mask] = a[mask] + b[mask]
    return out


def _exchange(t: torch.Tensor, peer: int, group) -> torch.Tensor:
    recv = torch.empty_like(t)
    ops = [dist.P2POp(dist.isend, t, peer, group), dist.P2POp(dist.irecv, recv, peer, group)]
    # lower rank sends first for backends that pair ops in order
    if dist.get_rank() > peer:
        ops.reverse()
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return recv


def adasum_allreduce_(flat: torch.Tensor, segments: Sequence[tuple[int, int]] | None = None,
                      ranks: Sequence[int] | None = None, group=None) -> torch.Tensor:
    """In-place flat Adasum over ``ranks`` (global ranks, default: the whole world)."""
    world = dist.get_world_size()
    ranks = list(range(world)) if ranks is None else list(ranks)
    me = dist.get_rank()
    if me not in ranks:
        raise ValueError("adasum_allreduce_: caller not in rank list")
    n = len(ranks)
    if n == 1:
        return flat
    pos = ranks.index(me)
    p2 = 1
    while p2 * 2 <= n:
        p2 *= 2
    work = flat
    # Fold the ranks beyond the largest power of two into their partners.
    if pos >= p2:
        dist.send(work.contiguous(), ranks[pos - p2], group=group)
        dist.recv(flat, ranks[pos - p2], group=group)
        return flat
    if pos + p2 < n:
        extra = torch.empty_like(work)
        dist.recv(extra, ranks[pos + p2], group=group)
        work = adasum_pair(work, extra, segments)
    d = 1
    while d < p2:
        peer_pos = pos ^ d
        other = _exchange(work.contiguous(), ranks[peer_pos], group)
        work = adasum_pair(work, other, segments) if pos < peer_pos else adasum_pair(other, work, segments)
        d *= 2
    if pos + p2 < n:
        dist.send(work.contiguous(), ranks[pos + p2], group=group)
    flat.copy_(work)
    return flat


def adasum_reference(vectors: Sequence[torch.Tensor], segments=None) -> torch.Tensor:
    """Single-process oracle of the distributed reduction (same pairing tree)."""
    vs = [v.clone() for v in vectors]
    n = len(vs)
    p2 = 1
    while p2 * 2 <= n:
        p2 *= 2
    for pos in range(p2, n):
        vs[pos - p2] = adasum_pair(vs[pos - p2], vs[pos], segments)
    vs = vs[:p2]
    d = 1
    while d < p2:
        nxt = list(vs)
        for pos in range(p2):
            peer = pos ^ d
            lo, hi = (pos, peer) if pos < peer else (peer, pos)
            nxt[pos] = adasum_pair(vs[lo], vs[hi], segments)
        vs = nxt
        d *= 2
    return vs[0]
