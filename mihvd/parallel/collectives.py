"""Tensor collectives with Horovod semantics (``hvd.allreduce / allgather / broadcast / alltoall /
reducescatter``, their grouped and ``_async`` forms, sparse allreduce, ``synchronize`` and ``poll``).

On GPUs over RCCL (world size > 1, or the collectives forced on) each world-level call is one
RCCL collective on the framework-owned communicator of :class:`BucketPlane` (NativeComm on its own
high-priority stream, the same one DistributedOptimizer's buckets use), ordered after the caller's
stream by an event; the handle's wait orders the caller's stream after it (no host block). Process
sets, host tensors, gloo, a running negotiation engine and the all-ranks fallback (the plane could
not be created) use the process group. Async calls return an integer handle; the native stall
inspector tracks every outstanding handle and the native timeline records a span per collective.
"""
from __future__ import annotations

import itertools
import threading
from typing import Any, Sequence

import torch
import torch.distributed as dist

from .. import basics
from ..basics import ReduceOp
from .compression import Compression, hip_pack, hip_pack_ok, hip_unpack

_handles: dict[int, "_Handle"] = {}
_hlock = threading.Lock()
_next = itertools.count(1)


class _Handle:
    __slots__ = ("work", "output", "post", "stall_id", "name", "done", "t0")

    def __init__(self, work, output, post, name):
        self.work = work
        self.output = output
        self.post = post
        self.name = name
        self.done = False
        ctx = basics._ctx
        self.stall_id = ctx.stall.submit(name) if ctx.stall is not None else None
        self.t0 = ctx.timeline.now_us() if ctx.timeline is not None else None


def _register(work, output, post, name) -> int:
    h = next(_next)
    handle = _Handle(work, output, post, name)
    with _hlock:
        _handles[h] = handle
    if basics._ctx.config is not None and basics._ctx.config.debug_sync:
        # serialized bisection mode: every collective completes before the call returns
        _finish(handle)
        if basics._ctx.device.type == "cuda":
            torch.cuda.synchronize()
    return h


def _finish(h: "_Handle"):
    if h.done:
        return h.output
    works = h.work if isinstance(h.work, (list, tuple)) else [h.work]
    for w in works:
        if w is not None:
            w.wait()
    if h.post is not None:
        h.output = h.post(h.output)
    h.done = True
    ctx = basics._ctx
    if h.stall_id is not None and ctx.stall is not None:
        ctx.stall.complete(h.stall_id)
    if h.t0 is not None and ctx.timeline is not None:
        kind = h.name.split(".", 1)[0].upper()
        ctx.timeline.complete(h.name, kind, 1, h.t0, ctx.timeline.now_us() - h.t0)
    return h.output


def synchronize(handle: int):
    """Wait for an async collective and return its output tensor."""
    with _hlock:
        h = _handles.pop(handle, None)
    if h is None:
        raise ValueError(f"unknown or already synchronized handle {handle}")
    return _finish(h)


def poll(handle: int) -> bool:
    with _hlock:
        h = _handles.get(handle)
    if h is None:
        raise ValueError(f"unknown handle {handle}")
    if h.done:
        return True
    works = h.work if isinstance(h.work, (list, tuple)) else [h.work]
    return all(w is None or w.is_completed() for w in works)


class _Children:
    """Work object of a handle built from other handles (grouped / sparse forms): ``poll`` on
    the parent reports completion only when every child collective has completed."""

    def __init__(self, handles):
        self.handles = list(handles)

    def is_completed(self) -> bool:
        with _hlock:
            live = [c for c in self.handles if c in _handles]  # absent: already synchronized
        return all(poll(c) for c in live)

    def wait(self):
        pass  # the parent's post() synchronizes the children in order


def _drain_all():
    with _hlock:
        hs = list(_handles.items())
        _handles.clear()
    for _, h in hs:
        try:
            _finish(h)
        except Exception:
            pass


def _torch_op(op: ReduceOp):
    return {
        ReduceOp.Sum: dist.ReduceOp.SUM,
        ReduceOp.Average: dist.ReduceOp.SUM,
        ReduceOp.Min: dist.ReduceOp.MIN,
        ReduceOp.Max: dist.ReduceOp.MAX,
        ReduceOp.Product: dist.ReduceOp.PRODUCT,
    }[op]


def _resolve_op(average, op):
    if op is not None and average is not None:
        raise ValueError("pass either op= or the deprecated average=, not both")
    if op is None:
        op = ReduceOp.Average if (average is None or average) else ReduceOp.Sum
    return ReduceOp(op)


def _group(process_set=None):
    from ..process_sets import resolve

    return resolve(process_set)


def _group_size(group) -> int:
    return dist.get_world_size(group) if group is not None else basics.size()


# ------------------------------------------------------------------------------------------ #
# allreduce
# ------------------------------------------------------------------------------------------ #
def _allreduce_impl(tensor, out, name, op, compression, prescale_factor, postscale_factor, group,
                    segments=None, async_op=True, wire_buf=None, plane=None):
    """``plane``: a :class:`BucketPlane` to run the collective on (DistributedOptimizer's buckets),
    instead of the engine / process group; it also runs at size 1 (forced collectives)."""
    ctx = basics._require()
    op = ReduceOp(op)
    n = _group_size(group)
    if plane is None and op != ReduceOp.Adasum:
        plane = _api_plane(group, tensor)
    if op == ReduceOp.Adasum:
        if out is not tensor:
            out.copy_(tensor)
        if prescale_factor != 1.0:
            out.mul_(prescale_factor)

        def run_adasum(out=out):
            adasum_dispatch_(out, segments)
            if postscale_factor != 1.0:
                out.mul_(postscale_factor)

        if ctx.engine is not None and n > 1:
            work = ctx.engine.collective(f"allreduce.{name}", "adasum", f"{out.dtype}|{tuple(out.shape)}", run_adasum)
            return _register(work, out, None, f"allreduce.{name}")
        run_adasum()
        return _register(None, out, None, f"allreduce.{name}")
    if hip_pack_ok(compression, tensor) and out.is_contiguous():
        # fused HIP pack (cast + prescale) -> collective on the 16-bit wire -> unpack (cast + scale);
        # at size 1 the wire round trip still runs (Horovod compresses at any size)
        wire = hip_pack(compression, tensor, prescale_factor, out=wire_buf)
        scale = postscale_factor / n if op == ReduceOp.Average else postscale_factor
        if plane is not None:
            work = plane.allreduce(wire, op)
        elif n == 1 and not getattr(ctx.engine, "world_one", False):
            work = None
        else:
            work = _engine_allreduce(ctx, f"allreduce.{name}", wire, _torch_op(op), group, ("hip-pack",))
        return _register(work, out, lambda _o, wire=wire, out=out, scale=scale: hip_unpack(wire, out, scale),
                         f"allreduce.{name}")
    wire, cctx = compression.compress(tensor)
    if wire is tensor and out is not tensor:
        out.copy_(tensor)
        wire = out
    if prescale_factor != 1.0:
        wire.mul_(prescale_factor)
    if plane is not None:
        work = plane.allreduce(wire, op)
    elif n == 1 and not getattr(ctx.engine, "world_one", False):
        work = None
    else:
        work = _engine_allreduce(ctx, f"allreduce.{name}", wire, _torch_op(op), group, ())
    scale = postscale_factor / n if op == ReduceOp.Average else postscale_factor

    def post(_o, wire=wire, cctx=cctx, out=out, scale=scale):
        res = compression.decompress(wire, cctx)
        if res is not out:
            out.copy_(res)
        if scale != 1.0:
            out.mul_(scale)
        return out

    return _register(work, out, post, f"allreduce.{name}")


class _PlaneWork:
    """Completion of a bucket collective on the plane's stream: ``wait()`` orders the caller's
    current stream behind it (no host block, like a process-group work object on RCCL), so it is
    also valid inside a HIP graph capture (the event becomes a graph dependency)."""

    __slots__ = ("ev", "device")

    def __init__(self, ev, device):
        self.ev = ev
        self.device = device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.ev)

    def is_completed(self) -> bool:
        return self.ev.query()


class BucketPlane:
    """DistributedOptimizer's gradient-bucket data plane on a framework-owned RCCL communicator
    ("called directly ... not through torch.distributed's ProcessGroup"; the
    reference's per-step allreduce is horovod/tensorflow_mnist.py:133). Each bucket's allreduce is
    enqueued on one dedicated high-priority HIP stream, ordered after the producing backward kernels
    by an event; the optimizer's ``synchronize()`` makes its stream wait for the bucket's completion
    event. The optimizer releases buckets strictly in order, so every rank issues the same
    collectives in the same order on the one stream -- no negotiation needed (the negotiated C++
    engine, MIHVD_ENGINE=native, is the path for named collectives that ranks may issue in
    different orders). Collective to construct: every rank of the world."""

    _OPS = {ReduceOp.Sum: "sum", ReduceOp.Average: "sum", ReduceOp.Min: "min", ReduceOp.Max: "max",
            ReduceOp.Product: "prod"}

    def __init__(self, device: torch.device):
        from .rccl import NativeComm

        self.device = device
        self.comm = NativeComm(device=device)
        self.stream = torch.cuda.Stream(device=device, priority=-1)
        self.launched = 0
        self.counts: dict[str, int] = {}  # collectives issued per kind (the public API's routing test)

    def _run(self, kind: str, fn) -> _PlaneWork:
        """``fn()`` on the plane's stream, ordered after everything the caller's stream queued so far
        (the inputs are complete there); the work's wait() orders the caller's stream after it."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            fn()
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.launched += 1
        self.counts[kind] = self.counts.get(kind, 0) + 1
        return _PlaneWork(ev, self.device)

    def allreduce(self, wire: torch.Tensor, op: ReduceOp) -> _PlaneWork:
        return self._run("allreduce", lambda: self.comm.all_reduce_(wire, self._OPS[op]))

    # the public collective API (hvd.broadcast / allgather / reducescatter / alltoall) on the same
    # communicator and stream: every rank issues them in program order, like the bucket allreduces
    def broadcast(self, t: torch.Tensor, root: int) -> _PlaneWork:
        return self._run("broadcast", lambda: self.comm.broadcast_(t, root))

    def allgather(self, out: torch.Tensor, inp: torch.Tensor) -> _PlaneWork:
        return self._run("allgather", lambda: self.comm.all_gather_into(out, inp))

    def reducescatter(self, out: torch.Tensor, inp: torch.Tensor, op: ReduceOp) -> _PlaneWork:
        return self._run("reducescatter", lambda: self.comm.reduce_scatter(out, inp, self._OPS[op]))

    def alltoall(self, out: torch.Tensor, inp: torch.Tensor, scnt, soff, rcnt, roff) -> _PlaneWork:
        return self._run("alltoall", lambda: self.comm.all_to_all_v(out, inp, scnt, soff, rcnt, roff))

    def close(self, abort: bool = False):
        self.comm.close(abort=abort)


def plane_wanted(world: int | None = None) -> bool:
    """Whether DistributedOptimizer's buckets go through :class:`BucketPlane`: RCCL backend, a GPU,
    ``MIHVD_COMM`` not ``torch``, and collectives (size > 1, or ``MIHVD_FORCE_COLLECTIVES=1``)."""
    import os

    from .rccl import env_mode

    ctx = basics._require()
    world = basics.size() if world is None else world
    forced = os.environ.get("MIHVD_FORCE_COLLECTIVES") == "1"
    return (ctx.backend == "nccl" and ctx.device is not None and ctx.device.type == "cuda" and env_mode() == "native"
            and (world > 1 or forced))


def bucket_plane():
    """The world's :class:`BucketPlane`, created on first use (collective: call on every rank, e.g.
    from every rank's DistributedOptimizer constructor), or None where :func:`plane_wanted` is
    false or the communicator cannot be created (then every rank falls back to the process group)."""
    ctx = basics._require()
    if ctx.plane is not None:
        return ctx.plane
    if not plane_wanted():
        return None
    plane, err = None, None
    try:
        plane = BucketPlane(ctx.device)
    except Exception as e:  # pragma: no cover - depends on the RCCL build
        err = e
    # every rank must use the same communicator: any failure moves all to the process group
    flag = torch.tensor([0 if plane is not None else 1], device=ctx.device)
    dist.all_reduce(flag)
    if int(flag.item()) != 0:
        if plane is not None:
            plane.close()
        import warnings

        warnings.warn(f"mihvd: native RCCL bucket plane unavailable ({err!r}); using the process group")
        return None
    ctx.plane = plane
    return plane


def _api_plane(group, *tensors):
    """The framework-owned communicator for a public collective (``hvd.allreduce`` outside
    DistributedOptimizer, ``broadcast*``, ``allgather*``, ``reducescatter``, ``alltoall``): the whole
    world, device tensors, the RCCL backend with ``MIHVD_COMM=native``, no negotiation engine (which
    orders named collectives itself). Otherwise None: the process group (sub-groups, gloo, the
    fallback every rank takes together when the plane cannot be created)."""
    if group is not None and group is not dist.group.WORLD:
        return None
    ctx = basics._ctx
    if ctx.engine is not None or not tensors or not all(t.is_cuda for t in tensors):
        return None
    if not plane_wanted():
        return None
    return bucket_plane()


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _engine_allreduce(ctx, name, wire, torch_op, group, fuse_extra):
    """Negotiated (launched by the engine thread in an order every rank agrees on, possibly fused)
    when an engine runs and the call is not being captured into a HIP graph; else on the process
    group. The native engine declines what it does not handle (sub-groups, other ops)."""
    if ctx.engine is not None and not _capturing():
        work = ctx.engine.allreduce(name, wire, torch_op, group, fuse_extra=fuse_extra)
        if work is not None:
            return work
    return dist.all_reduce(wire, op=torch_op, group=group, async_op=True)


def adasum_dispatch_(flat: torch.Tensor, segments=None, comm=None):
    """Adasum with Horovod-GPU semantics: hierarchical (average within node, Adasum across nodes)
    on the RCCL data plane, flat Adasum on gloo or when MIHVD_ADASUM_FLAT=1. On RCCL the world-level
    parts run on a framework-owned communicator (``comm``, else the bucket plane's): the node-local
    average when the node is the world, and flat Adasum as vector halving / distance doubling over
    ncclSend/ncclRecv (adasum.adasum_vhdd_) -- no host wait, capturable in a HIP graph. The
    cross-node Adasum of the hierarchical form runs over the cross-node process group."""
    from .adasum import adasum_allreduce_

    ctx = basics._require()
    topo = ctx.topology
    if comm is None and flat.is_cuda and ctx.backend == "nccl":
        plane = bucket_plane()
        comm = plane.comm if plane is not None else None
        if plane is not None:
            plane.launched += 1
    hierarchical = (ctx.backend == "nccl" and not ctx.config.adasum_flat and topo.local_size > 1
                    and ctx.local_group is not None)
    if not hierarchical:
        return adasum_allreduce_(flat, segments, comm=comm if comm is not None and comm.world == topo.size else None)
    if comm is not None and topo.cross_size == 1 and comm.world == topo.size:
        comm.all_reduce_(flat)  # the node is the world: the local average on the framework's communicator
    else:
        dist.all_reduce(flat, group=ctx.local_group)
    flat.div_(topo.local_size)
    if topo.cross_size > 1:
        ranks = list(range(topo.local_rank, topo.size, topo.local_size))
        adasum_allreduce_(flat, segments, ranks=ranks, group=ctx.cross_group)
    return flat


def allreduce_async(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0,
                    compression=Compression.none, process_set=None) -> int:
    op = _resolve_op(average, op)
    out = torch.empty_like(tensor)
    return _allreduce_impl(tensor, out, name or "tensor", op, compression, prescale_factor, postscale_factor,
                           _group(process_set))


def allreduce_async_(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0,
                     compression=Compression.none, process_set=None) -> int:
    op = _resolve_op(average, op)
    return _allreduce_impl(tensor, tensor, name or "tensor", op, compression, prescale_factor, postscale_factor,
                           _group(process_set))


def allreduce(tensor, average=None, name=None, compression=Compression.none, op=None, prescale_factor=1.0,
              postscale_factor=1.0, process_set=None):
    return synchronize(allreduce_async(tensor, average, name, op, prescale_factor, postscale_factor, compression,
                                       process_set))


def allreduce_(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0,
               process_set=None):
    return synchronize(allreduce_async_(tensor, average, name, op, prescale_factor, postscale_factor,
                                        process_set=process_set))


def _grouped_allreduce_async(tensors, op, name, compression, prescale_factor, postscale_factor, process_set,
                             inplace: bool) -> int:
    """One flat buffer and one collective per dtype; the handle's output is the list of results
    (views of the flat buffers, or the input tensors themselves when ``inplace``)."""
    tensors = list(tensors)
    by_dtype: dict[torch.dtype, list[int]] = {}
    for i, t in enumerate(tensors):
        by_dtype.setdefault(t.dtype, []).append(i)
    parts = []
    for dt, idxs in by_dtype.items():
        flat = torch.cat([tensors[i].reshape(-1) for i in idxs])
        segs, off = [], 0
        for i in idxs:
            segs.append((off, off + tensors[i].numel()))
            off += tensors[i].numel()
        h = _allreduce_impl(flat, flat, name or "grouped", op, compression, prescale_factor, postscale_factor,
                            _group(process_set), segments=segs)
        parts.append((h, idxs, segs))

    def post(_o, parts=parts):
        outs: list[Any] = [None] * len(tensors)
        for h, idxs, segs in parts:
            flat = synchronize(h)
            for i, (s, e) in zip(idxs, segs):
                outs[i] = flat[s:e].view_as(tensors[i])
                if inplace:
                    tensors[i].copy_(outs[i])
                    outs[i] = tensors[i]
        return outs

    return _register(_Children(h for h, _, _ in parts), None, post, f"grouped_allreduce.{name or 'grouped'}")


def grouped_allreduce_async(tensors: Sequence[torch.Tensor], average=None, name=None, op=None,
                            prescale_factor=1.0, postscale_factor=1.0, compression=Compression.none,
                            process_set=None) -> int:
    return _grouped_allreduce_async(tensors, _resolve_op(average, op), name, compression, prescale_factor,
                                    postscale_factor, process_set, inplace=False)


def grouped_allreduce_async_(tensors: Sequence[torch.Tensor], average=None, name=None, op=None,
                             prescale_factor=1.0, postscale_factor=1.0, process_set=None) -> int:
    return _grouped_allreduce_async(tensors, _resolve_op(average, op), name, Compression.none, prescale_factor,
                                    postscale_factor, process_set, inplace=True)


def grouped_allreduce(tensors: Sequence[torch.Tensor], average=None, name=None, compression=Compression.none,
                      op=None, prescale_factor=1.0, postscale_factor=1.0, process_set=None):
    """Fused allreduce of many tensors: one flat buffer per dtype, one collective each."""
    return synchronize(grouped_allreduce_async(tensors, average, name, op, prescale_factor, postscale_factor,
                                               compression, process_set))


def grouped_allreduce_(tensors: Sequence[torch.Tensor], average=None, name=None, op=None, prescale_factor=1.0,
                       postscale_factor=1.0, process_set=None):
    return synchronize(grouped_allreduce_async_(tensors, average, name, op, prescale_factor, postscale_factor,
                                                process_set))


def sparse_allreduce_async(tensor: torch.Tensor, name=None, op=ReduceOp.Average, process_set=None) -> int:
    """Allreduce of a sparse COO tensor (Horovod's ``sparse_allreduce_async``, used for
    ``sparse_as_dense=False`` embedding gradients): every rank's indices and values are
    all-gathered and summed into one coalesced tensor (``Average`` divides by the group size)."""
    op = ReduceOp(op)
    if op not in (ReduceOp.Average, ReduceOp.Sum):
        raise ValueError("sparse_allreduce supports Average and Sum")
    t = tensor.coalesce()
    hi = allgather_async(t.indices().t().contiguous(), name=f"{name or 'sparse'}.indices", process_set=process_set)
    hv = allgather_async(t.values().contiguous(), name=f"{name or 'sparse'}.values", process_set=process_set)
    n = _group_size(_group(process_set))

    def post(_o, hi=hi, hv=hv, shape=t.shape):
        idx = synchronize(hi).t()
        val = synchronize(hv)
        if op == ReduceOp.Average:
            val = val / n
        return torch.sparse_coo_tensor(idx, val, shape).coalesce()

    return _register(_Children((hi, hv)), None, post, f"sparse_allreduce.{name or 'sparse'}")


# ------------------------------------------------------------------------------------------ #
# broadcast / allgather / alltoall / reducescatter
# ------------------------------------------------------------------------------------------ #
def _flush_engine():
    """Direct (non-negotiated) collectives first wait until every negotiated one was launched."""
    ctx = basics._ctx
    if ctx.engine is not None:
        ctx.engine.flush()


def broadcast_async_(tensor, root_rank, name=None, process_set=None) -> int:
    ctx = basics._require()
    group = _group(process_set)
    name = f"broadcast.{name or 'tensor'}"
    plane = _api_plane(group, tensor) if tensor.is_contiguous() else None
    if plane is not None:  # (also at world 1 with the collectives forced on)
        work = plane.broadcast(tensor, root_rank)
    elif _group_size(group) == 1:
        work = None
    elif ctx.engine is not None:
        work = ctx.engine.collective(name, "broadcast", f"{tensor.dtype}|{tuple(tensor.shape)}|{root_rank}",
                                     lambda: dist.broadcast(tensor, src=root_rank, group=group, async_op=True))
    else:
        work = dist.broadcast(tensor, src=root_rank, group=group, async_op=True)
    return _register(work, tensor, None, name)


def broadcast_async(tensor, root_rank, name=None, process_set=None) -> int:
    out = tensor.clone()
    return broadcast_async_(out, root_rank, name, process_set)


def broadcast(tensor, root_rank, name=None, process_set=None):
    return synchronize(broadcast_async(tensor, root_rank, name, process_set))


def broadcast_(tensor, root_rank, name=None, process_set=None):
    return synchronize(broadcast_async_(tensor, root_rank, name, process_set))


def allgather_async(tensor, name=None, process_set=None) -> int:
    """Concatenate every rank's tensor along dim 0 (first dimensions may differ)."""
    ctx = basics._require()
    group = _group(process_set)
    n = _group_size(group)
    name = f"allgather.{name or 'tensor'}"
    t = tensor.contiguous()
    if t.dim() == 0:
        t = t.view(1)
    plane = _api_plane(group, t)
    if plane is not None:
        # dim 0 may differ per rank: the sizes first (one 8-byte all-gather on the plane, read on
        # the host), then every rank's rows padded to the largest
        dim0 = torch.tensor([t.shape[0]], dtype=torch.long, device=t.device)
        sizes_dev = torch.empty(n, dtype=torch.long, device=t.device)
        plane.allgather(sizes_dev, dim0).wait()
        sizes = [int(v) for v in sizes_dev.tolist()]
        mx = max(sizes)
        if mx != t.shape[0]:
            t = torch.cat([t, torch.zeros((mx - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)])
        full = torch.empty((n * mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        work = plane.allgather(full, t)

        def post_plane(_o, full=full, sizes=sizes, mx=mx):
            if all(sz == mx for sz in sizes):
                return full
            return torch.cat([full[i * mx:i * mx + sz] for i, sz in enumerate(sizes)])

        return _register(work, None, post_plane, name)
    if n == 1:
        return _register(None, tensor.clone(), None, name)
    res: dict = {}

    def launch(t=t):
        dim0 = torch.tensor([t.shape[0]], dtype=torch.long, device=t.device)
        sizes = [torch.empty_like(dim0) for _ in range(n)]
        dist.all_gather(sizes, dim0, group=group)
        sizes = [int(s.item()) for s in sizes]
        mx = max(sizes)
        if mx != t.shape[0]:
            pad = torch.zeros((mx - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            t = torch.cat([t, pad])
        res["bufs"] = [torch.empty_like(t) for _ in range(n)]
        res["sizes"] = sizes
        return dist.all_gather(res["bufs"], t, group=group, async_op=True)

    if ctx.engine is not None:
        # dim 0 may differ across ranks: the signature carries only dtype and trailing dims
        work = ctx.engine.collective(name, "allgather", f"{t.dtype}|{tuple(t.shape[1:])}", launch)
    else:
        work = launch()

    def post(_o, res=res):
        return torch.cat([b[:s] for b, s in zip(res["bufs"], res["sizes"])])

    return _register(work, None, post, name)


def allgather(tensor, name=None, process_set=None):
    return synchronize(allgather_async(tensor, name, process_set))


def grouped_allgather_async(tensors: Sequence[torch.Tensor], name=None, process_set=None) -> int:
    """``hvd.grouped_allgather_async``: every tensor all-gathered along dim 0 (first dims may
    differ per rank); the handle's output is the list of results in input order."""
    hs = [allgather_async(t, f"{name or 'grouped'}.{i}", process_set) for i, t in enumerate(tensors)]

    def post(_o, hs=hs):
        return [synchronize(h) for h in hs]

    return _register(_Children(hs), None, post, f"grouped_allgather.{name or 'grouped'}")


def grouped_allgather(tensors: Sequence[torch.Tensor], name=None, process_set=None):
    return synchronize(grouped_allgather_async(tensors, name, process_set))


def alltoall(tensor, splits=None, name=None, process_set=None):
    """Scatter slices of dim 0 to every rank and gather what they send back (``hvd.alltoall``).
    Returns ``(output, received_splits)``."""
    basics._require()
    _flush_engine()
    group = _group(process_set)
    n = _group_size(group)
    if splits is None:
        if tensor.shape[0] % n:
            raise ValueError("alltoall: first dimension must divide the world size when splits is None")
        splits = [tensor.shape[0] // n] * n
    splits = [int(s) for s in (splits.tolist() if torch.is_tensor(splits) else splits)]
    plane = _api_plane(group, tensor)
    if plane is not None:
        t = tensor.contiguous()
        row = 1
        for d in t.shape[1:]:
            row *= int(d)
        send_counts = torch.tensor(splits, dtype=torch.long, device=t.device)
        recv_counts = torch.empty_like(send_counts)
        ones = [1] * n
        offs = list(range(n))
        plane.alltoall(recv_counts, send_counts, ones, offs, ones, offs).wait()
        rsplits = [int(x) for x in recv_counts.tolist()]
        out = torch.empty((sum(rsplits),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        soff = [sum(splits[:j]) * row for j in range(n)]
        roff = [sum(rsplits[:j]) * row for j in range(n)]
        plane.alltoall(out.view(-1), t.view(-1), [c * row for c in splits], soff, [c * row for c in rsplits],
                       roff).wait()
        return out, torch.tensor(rsplits)
    if n == 1:
        return tensor.clone(), torch.tensor(splits)
    send_counts = torch.tensor(splits, dtype=torch.long, device=tensor.device)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    rsplits = [int(x) for x in recv_counts.tolist()]
    out = torch.empty((sum(rsplits),) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    if basics.backend() == "gloo":
        # gloo has no uneven all_to_all_single for every dtype: emulate with point-to-point.
        ins = list(torch.split(tensor.contiguous(), splits))
        outs = list(torch.split(out, rsplits))
        ops = []
        me = dist.get_rank(group) if group is not None else basics.rank()
        for p in range(n):
            if p == me:
                outs[p].copy_(ins[p])
                continue
            peer = dist.get_global_rank(group, p) if group is not None else p  # P2POp takes global ranks
            if ins[p].numel():
                ops.append(dist.P2POp(dist.isend, ins[p].contiguous(), peer, group))
            if outs[p].numel():
                ops.append(dist.P2POp(dist.irecv, outs[p], peer, group))
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
    else:
        dist.all_to_all_single(out, tensor.contiguous(), rsplits, splits, group=group)
    return out, torch.tensor(rsplits)


def alltoall_async(tensor, splits=None, name=None, process_set=None) -> int:
    """``hvd.alltoall_async``: the exchange runs at once (its split negotiation is itself a
    collective); ``synchronize`` returns ``(output, received_splits)``."""
    res = alltoall(tensor, splits, name, process_set)
    return _register(None, res, None, f"alltoall.{name or 'tensor'}")


def reducescatter_async(tensor, op=ReduceOp.Average, name=None, process_set=None) -> int:
    return _register(None, reducescatter(tensor, op, name, process_set), None, f"reducescatter.{name or 'tensor'}")


def grouped_reducescatter(tensors: Sequence[torch.Tensor], op=ReduceOp.Average, name=None, process_set=None):
    """Reduce-scatter of several tensors (each split along its own dim 0)."""
    return [reducescatter(t, op, f"{name or 'grouped'}.{i}", process_set) for i, t in enumerate(tensors)]


def grouped_reducescatter_async(tensors: Sequence[torch.Tensor], op=ReduceOp.Average, name=None,
                                process_set=None) -> int:
    return _register(None, grouped_reducescatter(tensors, op, name, process_set), None,
                     f"grouped_reducescatter.{name or 'grouped'}")


def reducescatter(tensor, op=ReduceOp.Average, name=None, process_set=None):
    """Reduce across ranks, then return this rank's dim-0 slice (``hvd.reducescatter``)."""
    basics._require()
    _flush_engine()
    group = _group(process_set)
    n = _group_size(group)
    op = ReduceOp(op)
    t = tensor.contiguous()
    plane = _api_plane(group, t) if op in BucketPlane._OPS else None
    if plane is None and n == 1:
        return tensor.clone()
    dim0 = t.shape[0]
    base, rem = divmod(dim0, n)
    counts = [base + (1 if i < rem else 0) for i in range(n)]
    me = dist.get_rank(group) if group is not None else basics.rank()
    if plane is not None:
        if rem == 0:
            out = torch.empty((counts[me],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            plane.reducescatter(out, t, op).wait()
        else:  # uneven blocks: the whole reduction, then this rank's rows
            full = t.clone()
            plane.allreduce(full, op).wait()
            start = sum(counts[:me])
            out = full[start:start + counts[me]].clone()
        if op == ReduceOp.Average:
            out.div_(n)
        return out
    if rem == 0 and basics.backend() == "nccl":
        out = torch.empty((counts[me],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, t, op=_torch_op(op), group=group)
    else:
        full = t.clone()
        dist.all_reduce(full, op=_torch_op(op), group=group)
        start = sum(counts[:me])
        out = full[start:start + counts[me]].clone()
    if op == ReduceOp.Average:
        out.div_(n)
    return out


def barrier(process_set=None):
    basics._require()
    _flush_engine()
    if basics.size() > 1:
        if basics.backend() == "nccl":
            dist.barrier(device_ids=[basics.device().index])
        else:
            dist.barrier()


def join(device=-1) -> int:
    """Horovod ``join``: block until every rank arrives; returns the last rank to join."""
    basics._require()
    _flush_engine()
    t = torch.tensor([basics.rank()], dtype=torch.long, device=basics.device())
    if basics.size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def broadcast_object(obj, root_rank=0, name=None, process_set=None):
    basics._require()
    _flush_engine()
    if basics.size() == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=root_rank, group=_group(process_set),
                               device=basics.device() if basics.backend() == "nccl" else None)
    return lst[0]


def allgather_object(obj, name=None, process_set=None):
    basics._require()
    _flush_engine()
    if basics.size() == 1:
        return [obj]
    out = [None] * basics.size()
    dist.all_gather_object(out, obj, group=_group(process_set))
    return out
