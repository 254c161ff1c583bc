"""A framework-owned RCCL communicator (csrc/kernels/rccl_comm.cpp).

Horovod's native core owns its NCCL communicator and enqueues the step's fused allreduce
(horovod/tensorflow_mnist.py:133, hvd.DistributedOptimizer) on its own stream. :class:`NativeComm`
is that object here: rank 0 draws an ``ncclUniqueId``, the ranks exchange it over the bootstrap
process group, and every rank calls ``ncclCommInitRank`` through the librccl the process already
loaded (the same library torch's ProcessGroupNCCL uses). Its collectives enqueue straight onto the
caller's current HIP stream — the trainer's side stream, or a stream being captured into the step's
HIP graph — with no process-group work objects around them, and the communicator is registered
with the native health monitor (async-error polling → abort, csrc/runtime/health.cc).

The fused trainer's collectives use it by default (``MIHVD_COMM=native``); ``MIHVD_COMM=torch``
selects the process group's RCCL communicator instead, which is also the fallback when the
native communicator cannot be created. The process group then only carries the bootstrap (the
unique-id broadcast) and host-synchronised control traffic (initial broadcast, barriers), never a
collective inside the step's HIP graph — so torch's ProcessGroupNCCL watchdog never sees a
captured event.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .. import ops as _ops

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


def env_mode() -> str:
    """``MIHVD_COMM``: ``native`` (a framework-owned communicator, default) or ``torch`` (the
    process group's)."""
    v = os.environ.get("MIHVD_COMM", "native").strip().lower()
    return "torch" if v in ("torch", "pg", "0", "off") else "native"


class NativeComm:
    """Collective: every rank of ``group`` constructs it. Needs the nccl (RCCL) backend."""

    def __init__(self, group=None, device: torch.device | None = None):
        if not dist.is_initialized() or dist.get_backend(group) != "nccl":
            raise RuntimeError("NativeComm needs a process group on the nccl (RCCL) backend")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self._o = _ops.load()
        uid = [self._o.rccl_unique_id() if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(uid, src=src, group=group, device=device)
        with torch.cuda.device(device):
            self.handle = int(self._o.rccl_comm_init(uid[0], self.rank, self.world, device.index))
        self._closed = False
        self._attach_health()

    def _attach_health(self):
        from .. import basics

        mon = getattr(basics._ctx, "health", None)
        if mon is None:
            return
        try:
            mon.attach_rccl(int(self._o.rccl_comm_ptr(self.handle)), str(self._o.rccl_library_path()))
        except Exception:  # pragma: no cover - the monitor is best effort
            pass

    # every collective runs on the current HIP stream -----------------------------------------
    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        self._o.rccl_all_reduce_(self.handle, t, _OPS[op])
        return t

    def all_reduce_many_(self, ts, op: str = "sum"):
        """Several all-reduces as one RCCL group call."""
        self._o.rccl_all_reduce_many_(self.handle, list(ts), _OPS[op])

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """``out`` = concatenation over ranks of ``inp`` (``inp`` may be this rank's slice of ``out``)."""
        self._o.rccl_all_gather(self.handle, out, inp)
        return out

    def all_gather_many_into(self, outs, inps):
        """Several all-gathers as one RCCL group call (``inps[i]`` may be this rank's slice of
        ``outs[i]``: in place)."""
        self._o.rccl_all_gather_many(self.handle, list(outs), list(inps))

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> torch.Tensor:
        self._o.rccl_reduce_scatter(self.handle, out, inp, _OPS[op])
        return out

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """Block j of ``inp`` goes to rank j; block j of ``out`` comes from rank j (equal blocks)."""
        self._o.rccl_all_to_all(self.handle, out, inp)
        return out

    def send_recv(self, send: torch.Tensor, recv: torch.Tensor, peer: int) -> torch.Tensor:
        """One pairwise exchange with ``peer`` (an RCCL group of one send and one receive)."""
        self._o.rccl_send_recv(self.handle, send, recv, int(peer))
        return recv

    def all_to_all_v(self, out: torch.Tensor, inp: torch.Tensor, scnt, soff, rcnt, roff) -> torch.Tensor:
        """Uneven all-to-all over flat element ranges (counts and offsets in elements, one per rank)."""
        self._o.rccl_all_to_all_v(self.handle, out, inp, [int(v) for v in scnt], [int(v) for v in soff],
                                  [int(v) for v in rcnt], [int(v) for v in roff])
        return out

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        self._o.rccl_broadcast_(self.handle, t, root)
        return t

    def nranks(self) -> int:
        """The communicator's size as RCCL reports it (ncclCommCount)."""
        return int(self._o.rccl_comm_count(self.handle))

    def user_rank(self) -> int:
        """This rank as RCCL reports it (ncclCommUserRank)."""
        return int(self._o.rccl_comm_user_rank(self.handle))

    def async_error(self) -> int:
        return int(self._o.rccl_async_error(self.handle))

    def close(self, abort: bool = False):
        if not self._closed:
            from .. import basics

            mon = getattr(basics._ctx, "health", None)
            if mon is not None:
                mon.detach_rccl(int(self._o.rccl_comm_ptr(self.handle)))
            if not abort:
                # a peer that died with a collective in flight would hold this wait forever: after a
                # failure the communicator is aborted (ncclCommAbort) without draining the device
                torch.cuda.synchronize(self.device)
            self._o.rccl_comm_destroy(self.handle, abort)
            self._closed = True

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            if not getattr(self, "_closed", True) and torch.cuda.is_initialized():
                self.close()
        except Exception:
            pass


__all__ = ["NativeComm", "env_mode"]
