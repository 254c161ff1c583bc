"""Adasum reduction (``hvd.Adasum``; reference: ``--use-adasum``, horovod/tensorflow_mnist.py:31-32,126-127,133).

Adasum combines two gradients scale-invariantly, per tensor (layer)::

    adasum(a, b) = (1 - a.b / (2|a|^2)) a + (1 - a.b / (2|b|^2)) b

and reduces N ranks by vector halving / distance doubling over point-to-point exchanges
(``adasum_vhdd_``: on MI355X each exchange is an RCCL ``ncclSend``/``ncclRecv`` pair over the xGMI
link between the two GPUs, on the framework-owned communicator). Non-power-of-two worlds first fold
the extra ranks into their partners and send the result back at the end.

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


# ------------------------------------------------------------------------------------------ #
# Vector-halving / distance-doubling (VHDD) Adasum over a transport
# ------------------------------------------------------------------------------------------ #
class PGTransport:
    """Pairwise exchanges and the small dot-product sums over the process group (gloo on the CPU, or
    the RCCL process group as the fallback). ``ranks``: the global ranks taking part, in order."""

    def __init__(self, ranks: Sequence[int] | None = None, group=None):
        world = dist.get_world_size()
        self.ranks = list(range(world)) if ranks is None else list(ranks)
        self.group = group
        self.size = len(self.ranks)
        self.pos = self.ranks.index(dist.get_rank())
        self.bytes_sent = 0

    def send_recv(self, send: torch.Tensor, recv: torch.Tensor, peer: int):
        ops = []
        if send.numel():
            ops.append(dist.P2POp(dist.isend, send.contiguous(), self.ranks[peer], self.group))
            self.bytes_sent += send.numel() * send.element_size()
        if recv.numel():
            ops.append(dist.P2POp(dist.irecv, recv, self.ranks[peer], self.group))
        if self.pos > peer:  # backends that pair operations in order: the lower position sends first
            ops.reverse()
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()

    def allreduce(self, t: torch.Tensor):
        dist.all_reduce(t, group=self.group)


class NativeTransport:
    """The same over the framework-owned RCCL communicator (mihvd/parallel/rccl.py NativeComm):
    ``ncclSend``/``ncclRecv`` in one group per exchange and ``ncclAllReduce`` of the dot products,
    all enqueued on the current stream with no host wait, so the whole reduction replays from a HIP
    graph."""

    def __init__(self, comm):
        self.comm = comm
        self.size = comm.world
        self.pos = comm.rank
        self.bytes_sent = 0

    def send_recv(self, send: torch.Tensor, recv: torch.Tensor, peer: int):
        self.bytes_sent += send.numel() * send.element_size()
        self.comm.send_recv(send, recv, peer)

    def allreduce(self, t: torch.Tensor):
        self.comm.all_reduce_(t)


def _split(lo: int, hi: int) -> int:
    """Midpoint of a range being halved (64-element aligned when the range is long enough)."""
    n = hi - lo
    if n >= 256:
        return lo + (n // 2) // 64 * 64
    return lo + n // 2


class _VHDDPlan:
    """Per (vector length, segments, position, size) tables of the halving schedule: the kept /
    given ranges per level and every level's segment table in the kept range's coordinates (the
    global segments clipped, so every rank of a group indexes the same S segments)."""

    def __init__(self, n: int, segments, pos: int, size: int, device):
        p2 = 1
        while p2 * 2 <= size:
            p2 *= 2
        self.p2 = p2
        self.levels = []
        offs, flags = _covering_offsets(segments, n)
        self.S = len(offs) - 1
        lo, hi = 0, n
        d = 1
        while d < p2 and pos < p2:
            mid = _split(lo, hi)
            low = (pos & d) == 0
            keep, give = ((lo, mid), (mid, hi)) if low else ((mid, hi), (lo, mid))
            a, b = keep
            loc = [min(max(o, a), b) - a for o in offs]
            tab = torch.tensor(loc + flags, dtype=torch.int64)
            max_len = max([e - s for s, e in zip(loc[:-1], loc[1:])] + [1])
            self.levels.append({"d": d, "parent": (lo, hi), "keep": keep, "give": give, "low": low,
                                "offs_host": (loc, flags), "offs": tab.to(device) if device.type == "cuda" else tab,
                                "max_len": max_len})
            lo, hi = keep
            d *= 2
        self.L = 0
        while (1 << self.L) < p2:
            self.L += 1
        self.dots = [torch.zeros(max(1, p2 // (2 << l)), self.S, 3, dtype=torch.float64, device=device)
                     for l in range(self.L)]
        self.recv = torch.empty((n + 1) // 2 + 64, dtype=torch.float32, device=device)


_VHDD_PLANS: dict = {}


def _dots_into(a, b, lv, out):
    """Per-segment (a.b, |a|^2, |b|^2) of this level's kept piece into out [S, 3] (fp64)."""
    if a.is_cuda and a.dtype == torch.float32:
        torch.ops.mihvd.segment_dots(a, b, lv["offs"], lv["max_len"], out)
        return
    loc, flags = lv["offs_host"]
    a64, b64 = a.double(), b.double()
    for i, (s, e) in enumerate(zip(loc[:-1], loc[1:])):
        if flags[i] or e <= s:
            continue
        x, y = a64[s:e], b64[s:e]
        out[i, 0] = torch.dot(x, y)
        out[i, 1] = torch.dot(x, x)
        out[i, 2] = torch.dot(y, y)


def _combine_into(a, b, lv, dots, out):
    """out = ca a + cb b per segment from the group's summed dots (plain sum on gap segments)."""
    if a.is_cuda and a.dtype == torch.float32:
        torch.ops.mihvd.adasum_combine(a, b, lv["offs"], lv["max_len"], dots, out)
        return
    loc, flags = lv["offs_host"]
    for i, (s, e) in enumerate(zip(loc[:-1], loc[1:])):
        if e <= s:
            continue
        if flags[i]:
            out[s:e] = a[s:e] + b[s:e]
            continue
        ab, aa, bb = (float(v) for v in dots[i])
        ca = (1.0 - ab / (2.0 * aa) if aa > 0 else 0.0) if bb > 0 else 1.0
        cb = (1.0 - ab / (2.0 * bb) if bb > 0 else 0.0) if aa > 0 else 1.0
        out[s:e] = a[s:e] * ca + b[s:e] * cb


def adasum_vhdd_(flat: torch.Tensor, segments: Sequence[tuple[int, int]] | None, transport) -> torch.Tensor:
    """In-place Adasum of ``flat`` over the transport's ranks by vector halving / distance doubling
    (Horovod's Adasum allreduce): at level d a rank exchanges half of its current
    range with the partner at distance 2^d (it keeps one half, the partner the other), the pair's
    per-tensor dot products are summed over the 2^(d+1) ranks holding pieces of the two vectors
    (one small allreduce: every group's sums in its own slot), and the kept half is combined; after
    log2(N) levels every rank holds 1/N of the result and the halves travel back in reverse order.
    Per rank about 2 S (N-1)/N bytes are sent instead of log2(N) S for whole-vector doubling. The
    pairing tree is adasum_reference's, so the result equals it to fp32 rounding of the dot sums.
    Ranks beyond the largest power of two fold into their partners first (whole vectors) and take
    part in the dot sums with zeros. Transports: NativeTransport (RCCL, graph-capturable) or
    PGTransport."""
    n_ranks, pos = transport.size, transport.pos
    if n_ranks == 1:
        return flat
    if segments is None:
        segments = [(0, flat.numel())]
    key = (flat.numel(), tuple(segments), pos, n_ranks, flat.device, flat.dtype)
    plan = _VHDD_PLANS.get(key)
    if plan is None:
        plan = _VHDD_PLANS[key] = _VHDDPlan(flat.numel(), segments, pos, n_ranks, flat.device)
        if plan.recv.dtype != flat.dtype:
            plan.recv = plan.recv.to(flat.dtype)
    p2 = plan.p2
    empty = flat[:0]
    if pos >= p2:  # an extra rank: fold into the partner, join the dot sums with zeros, take the result
        transport.send_recv(flat, empty, pos - p2)
        for l in range(plan.L):
            plan.dots[l].zero_()
            transport.allreduce(plan.dots[l])
        transport.send_recv(empty, flat, pos - p2)
        return flat
    if pos + p2 < n_ranks:  # take the extra rank's vector and combine the whole vector first
        extra = torch.empty_like(flat)
        transport.send_recv(empty, extra, pos + p2)
        flat.copy_(adasum_pair(flat, extra, segments))
    for l, lv in enumerate(plan.levels):
        (klo, khi), (glo, ghi) = lv["keep"], lv["give"]
        recv = plan.recv[:khi - klo]
        transport.send_recv(flat[glo:ghi], recv, pos ^ lv["d"])
        mine = flat[klo:khi]
        a, b = (mine, recv) if lv["low"] else (recv, mine)
        dots = plan.dots[l]
        dots.zero_()
        slot = dots[pos // (2 * lv["d"])]
        _dots_into(a, b, lv, slot)
        transport.allreduce(dots)
        _combine_into(a, b, lv, slot, mine)
    for lv in reversed(plan.levels):  # distance halving: the halves back to both partners
        (klo, khi), (glo, ghi) = lv["keep"], lv["give"]
        transport.send_recv(flat[klo:khi], flat[glo:ghi], pos ^ lv["d"])
    if pos + p2 < n_ranks:
        transport.send_recv(flat, empty, pos + p2)
    global last_bytes_sent
    last_bytes_sent = transport.bytes_sent
    return flat


last_bytes_sent = 0  # bytes this rank sent in the last adasum_vhdd_ (tests: the ~2 S (N-1)/N volume)


def adasum_allreduce_(flat: torch.Tensor, segments: Sequence[tuple[int, int]] | None = None,
                      ranks: Sequence[int] | None = None, group=None, comm=None) -> torch.Tensor:
    """In-place flat Adasum over ``ranks`` (global ranks, default: the whole world): VHDD over the
    framework-owned RCCL communicator ``comm`` (a NativeComm of the whole world) when given, else over
    the process group."""
    transport = NativeTransport(comm) if comm is not None else PGTransport(ranks, group)
    return adasum_vhdd_(flat, segments, transport)


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
