"""Process sets (Horovod ``hvd.ProcessSet``): collectives over a subset of the ranks.

    ps = hvd.ProcessSet([0, 2])           # or hvd.init(process_sets=[...]) / hvd.add_process_set
    hvd.add_process_set(ps)               # collective over the world (every rank calls it)
    if ps.included():
        hvd.allreduce(t, process_set=ps)  # Average divides by ps.size()

Each set owns a ``torch.distributed`` group (an RCCL communicator over those GPUs' xGMI links, or
gloo on the CPU). ``global_process_set`` is the world.
"""
from __future__ import annotations

import threading

import torch.distributed as dist

from . import basics

_lock = threading.Lock()
_sets: dict[int, "ProcessSet"] = {}
_next_id = 1


class ProcessSet:
    def __init__(self, ranks):
        self.ranks = sorted({int(r) for r in ranks}) if ranks is not None else None
        self.process_set_id: int | None = None
        self._group = None

    # Horovod API --------------------------------------------------------------------------
    def size(self) -> int:
        return len(self.ranks) if self.ranks is not None else basics.size()

    def rank(self) -> int:
        me = basics.rank()
        if self.ranks is None:
            return me
        return self.ranks.index(me) if me in self.ranks else -1

    def included(self) -> bool:
        return self.ranks is None or basics.rank() in self.ranks

    def __repr__(self):
        return f"ProcessSet(process_set_id={self.process_set_id}, ranks={self.ranks})"

    # internal -----------------------------------------------------------------------------
    @property
    def group(self):
        """The torch.distributed group (None = the world)."""
        if self.ranks is None:
            return None
        if self.process_set_id is None:
            raise ValueError(f"{self!r} has not been registered: call hvd.add_process_set() on every rank")
        if not self.included():
            raise ValueError(f"rank {basics.rank()} is not part of {self!r}")
        return self._group


global_process_set = ProcessSet(None)
global_process_set.process_set_id = 0


def add_process_set(process_set) -> ProcessSet:
    """Register a process set (a list of ranks or a ProcessSet). Collective: every rank calls it in
    the same order, as torch.distributed.new_group requires."""
    global _next_id
    basics._require()
    ps = process_set if isinstance(process_set, ProcessSet) else ProcessSet(process_set)
    if ps.ranks is None:
        return global_process_set
    if any(not 0 <= r < basics.size() for r in ps.ranks):
        raise ValueError(f"process set ranks {ps.ranks} outside the world of size {basics.size()}")
    with _lock:
        for other in _sets.values():
            if other.ranks == ps.ranks:
                raise ValueError(f"a process set with ranks {ps.ranks} already exists: {other!r}")
        ps._group = dist.new_group(ps.ranks)
        ps.process_set_id = _next_id
        _sets[_next_id] = ps
        _next_id += 1
    return ps


def remove_process_set(process_set: ProcessSet) -> bool:
    with _lock:
        if process_set.process_set_id in _sets:
            del _sets[process_set.process_set_id]
            if process_set._group is not None and process_set.included():
                dist.destroy_process_group(process_set._group)
            process_set._group = None
            process_set.process_set_id = None
            return True
    return False


def get_process_set_ids_and_ranks() -> dict[int, list[int]]:
    out = {0: list(range(basics.size()))}
    out.update({i: ps.ranks for i, ps in _sets.items()})
    return out


def _reset():
    """Forget every process set (their groups die with the world at shutdown)."""
    global _next_id
    with _lock:
        for ps in _sets.values():
            ps._group = None
            ps.process_set_id = None
        _sets.clear()
        _next_id = 1


def resolve(process_set):
    """Collective helper: ProcessSet | torch group | None -> torch group (None = world)."""
    if process_set is None or process_set is global_process_set:
        return None
    if isinstance(process_set, ProcessSet):
        return process_set.group
    return process_set  # already a torch.distributed group
