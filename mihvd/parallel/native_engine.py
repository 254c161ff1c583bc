"""The native collective engine (``csrc/kernels/engine.cpp``): Horovod's background loop in C++.

``MIHVD_ENGINE=native`` (opt-in) routes every asynchronous allreduce — the DistributedOptimizer's
bucket allreduces issued from gradient hooks, ``allreduce_async`` — through one C++ thread per
process that owns two framework RCCL communicators (:class:`mihvd.parallel.rccl.NativeComm`): a
control communicator for negotiation and a data communicator for the fused allreduces, each on its
own high-priority HIP stream. The thread is event-driven: it sleeps until a tensor is enqueued, then
negotiates readiness with one small RCCL allreduce of a per-slot count + signature-hash vector
(Horovod's bit-vector response cache, on the GPU), packs ready tensors into a persistent fusion
buffer (one batched pack kernel) up to ``HOROVOD_FUSION_THRESHOLD``, reduces, unpacks (one kernel)
and records a pooled completion event per request, without waiting for the data stream: the next
negotiation overlaps the previous cycle's collectives. ``HOROVOD_CYCLE_TIME`` only bounds how long
a rank whose work is partly ready waits before re-negotiating. The stall inspector reports
collectives that only some ranks reached (and negotiations peers never joined) and aborts after
``HOROVOD_STALL_SHUTDOWN_TIME_SECONDS``.

Ranks may enqueue tensors in different orders: slots are numbered from data every rank holds (the
sorted union of newly announced signature hashes, all-gathered), a collective runs only once every
rank enqueued its signature (name, dtype, size, op), and every rank derives the same launch order
from the same summed vector, so mismatched autograd schedules cannot deadlock or mismatch RCCL calls
(horovod/tensorflow_mnist.py:133 relies on this implicitly).

Non-allreduce collectives (broadcast, allgather, Adasum) keep running on the process group's
communicator in program order; collectives issued while a HIP graph is being captured bypass the
engine (a captured step is replayed, not negotiated).
"""
from __future__ import annotations

import threading

import torch
import torch.distributed as dist

from .. import ops as _ops

_OP_CODES = {dist.ReduceOp.SUM: 0, dist.ReduceOp.PRODUCT: 1, dist.ReduceOp.MAX: 2, dist.ReduceOp.MIN: 3}


class NativeWork:
    """Work handle of an engine allreduce: ``wait()`` blocks until the engine has enqueued the
    collective, then orders the caller's current stream after it (no host-device sync)."""

    __slots__ = ("_h", "_engine", "_done")

    def __init__(self, h: int, engine: "NativeEngine"):
        self._h = h
        self._engine = engine
        self._done = False

    def wait(self):
        if not self._done:
            self._engine._o.engine_wait(self._h)
            self._done = True
            self._engine._forget(self)
        return True

    def is_completed(self) -> bool:
        return self._done or bool(self._engine._o.engine_poll(self._h))


class NativeEngine:
    """Collective over the world: every rank constructs it (after the process group exists)."""

    def __init__(self, cfg, device: torch.device, comm=None, max_slots: int = 1024):
        from .rccl import NativeComm

        self._o = _ops.load()
        self.comm = comm if comm is not None else NativeComm(device=device)
        self.ctrl_comm = NativeComm(device=self.comm.device)  # negotiation, on its own stream
        self.world = self.comm.world
        # an engine started at world size 1 (MIHVD_ENGINE=native) still carries every allreduce, as
        # Horovod's does: the same negotiation / fusion / completion path as at N ranks
        self.world_one = self.world == 1
        self.fusion_threshold = int(cfg.fusion_threshold)
        warn = 0.0 if cfg.stall_check_disable else float(cfg.stall_check_s)
        self._o.engine_start(self.comm.handle, self.ctrl_comm.handle, self.fusion_threshold,
                             max(cfg.cycle_time_ms, 0.05) / 1000.0, warn, float(cfg.stall_shutdown_s), int(max_slots))
        self._lock = threading.Lock()
        self._outstanding: set = set()

    # the python Engine's interface (mihvd/parallel/engine.py), so collectives.py can use either
    def allreduce(self, name: str, wire: torch.Tensor, torch_op, group, fuse_extra=()):
        if group not in (None, dist.group.WORLD) or torch_op not in _OP_CODES or not wire.is_contiguous():
            return None  # not for the engine: the caller launches it on the process group
        w = NativeWork(int(self._o.engine_allreduce_async(wire, name, _OP_CODES[torch_op])), self)
        with self._lock:
            self._outstanding.add(w)
        return w

    def collective(self, name: str, kind: str, signature: str, launch):
        return launch()

    def _forget(self, w):
        with self._lock:
            self._outstanding.discard(w)

    def flush(self, timeout: float | None = None):
        with self._lock:
            pending = list(self._outstanding)
        for w in pending:
            w.wait()

    def stats(self) -> dict:
        c, n, t, fb, slots, stalls, wake, idle, ann = (int(x) for x in self._o.engine_stats())
        return {"cycles": c, "collectives": n, "tensors": t, "fused_bytes": fb, "slots": slots, "stall_warnings": stalls,
                "wakeups": wake, "idle_waits": idle, "announce_rounds": ann}

    def stop(self):
        self.flush()
        self._o.engine_stop()
        self.ctrl_comm.close()
        self.comm.close()


def plan(ctrl, world: int, hashes, nbytes, keys, threshold: int):
    """The engine's planning step on a summed control vector (CPU; for tests): returns
    (groups, partial) — lists of fused slot groups and the slots pending on only some ranks."""
    o = _ops.load()
    out = list(o.engine_plan(torch.as_tensor(ctrl, dtype=torch.int32), int(world), torch.as_tensor(hashes, dtype=torch.int64),
                             torch.as_tensor(nbytes, dtype=torch.int64), torch.as_tensor(keys, dtype=torch.int64),
                             int(threshold)))
    cut = out.index(-2)
    groups, cur = [], []
    for e in out[:cut]:
        if e == -1:
            groups.append(cur)
            cur = []
        else:
            cur.append(int(e))
    return groups, [int(s) for s in out[cut + 1:]]


def assign(gathered, world: int, assigned=()):
    """The engine's slot agreement on an all-gathered announce array (CPU; for tests): the hashes
    that get new slots, in the order every rank appends them."""
    o = _ops.load()
    return [int(h) & 0xFFFFFFFF for h in o.engine_assign(torch.as_tensor(gathered, dtype=torch.int64).to(torch.int32),
                                                         int(world), torch.as_tensor(list(assigned), dtype=torch.int64))]


def signature_hash(name: str, dtype_code: int, numel: int, op: int) -> int:
    return int(_ops.load().engine_signature_hash(f"{name}|{dtype_code}|{numel}|{op}"))


__all__ = ["NativeEngine", "NativeWork", "assign", "plan", "signature_hash"]
