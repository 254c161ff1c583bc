"""Elastic training: ``hvd.elastic.run`` / ``TorchState`` / ``ObjectState`` (Horovod Elastic).

The reference points at an elastic variant of its MPIJob (horovod/README.md:20-22)
but ships none. Here it is built on the framework's own control plane:

* ``mihvdrun --min-np M [--max-np N] [--respawn]`` is the elastic driver. It hosts the C++ store,
  gives every worker a stable ``MIHVD_WORKER_ID`` and publishes the membership of each
  *generation* in the store (``elastic/gen``, ``elastic/members/<g>`` = ``id@host,...`` in rank
  order). When a worker dies it publishes a new generation without it (or with a respawned
  replacement, ``--respawn``) as long as at least ``--min-np`` workers remain; below that the job
  is torn down with mpirun semantics.
* ``mihvd.init()`` in a worker (``MIHVD_ELASTIC=1``) derives rank/size from the newest generation
  that contains its id and builds the process group on a generation-scoped prefix of the store.
* ``@hvd.elastic.run`` wraps the training function: state is synchronised from rank 0 on entry;
  when a collective fails because a peer died (the driver has published a newer generation), the
  state is rolled back to the last ``commit()``, the world is re-formed and training resumes; when
  workers are added, ``commit()`` raises ``HostsUpdatedInterrupt`` on every rank at the same step
  (the check is one collective) and the world is re-formed without a rollback.
* GPU tensors keep their device: a worker always drives the GPU of its launch slot.
"""
from __future__ import annotations

import copy
import functools
import logging
import time

import torch

from . import basics

log = logging.getLogger("mihvd.elastic")


class HorovodInternalError(RuntimeError):
    """A collective failed because the set of workers changed (a peer died)."""


class HostsUpdatedInterrupt(RuntimeError):
    """Workers were added or removed; the world must be re-formed (raised by ``commit()``)."""

    def __init__(self, skip_sync: bool = False):
        super().__init__("hosts updated")
        self.skip_sync = skip_sync


# ------------------------------------------------------------------------------------------ #
# membership (worker side)
# ------------------------------------------------------------------------------------------ #
GEN_KEY = "elastic/gen"


def members_key(g: int) -> str:
    return f"elastic/members/{g}"


def parse_members(raw: bytes | str) -> list[tuple[int, str]]:
    s = raw.decode() if isinstance(raw, bytes) else raw
    out = []
    for item in filter(None, s.split(",")):
        wid, _, host = item.partition("@")
        out.append((int(wid), host or "localhost"))
    return out


def format_members(members: list[tuple[int, str]]) -> str:
    return ",".join(f"{w}@{h}" for w, h in members)


def current_generation(store) -> int:
    v = store.try_get(GEN_KEY, 0.0)
    return int(v) if v is not None else -1


def wait_for_membership(store, worker_id: int, after_gen: int, timeout_s: float):
    """Newest generation > after_gen that contains worker_id: (gen, rank, size, local_rank,
    local_size). Blocks (server-side parked reads) until the driver publishes one."""
    deadline = time.time() + timeout_s
    g = max(after_gen + 1, 0)
    while True:
        latest = current_generation(store)
        if latest >= g:
            g = latest  # skip straight to the newest generation
            members = parse_members(store.get(members_key(g)))
            ids = [w for w, _ in members]
            if worker_id in ids:
                rank = ids.index(worker_id)
                host = members[rank][1]
                same = [w for w, h in members if h == host]
                return g, rank, len(members), same.index(worker_id), len(same)
            g += 1
        left = deadline - time.time()
        if left <= 0:
            raise TimeoutError(f"worker {worker_id}: no elastic generation > {after_gen} includes it")
        store.try_get(members_key(g), min(left, 1.0))  # park until generation g appears


# ------------------------------------------------------------------------------------------ #
# state objects
# ------------------------------------------------------------------------------------------ #
class State:
    """Base class: ``commit / restore / sync / check_host_updates`` + reset callbacks."""

    def __init__(self):
        self._reset_callbacks = []
        self.commits = 0

    def register_reset_callbacks(self, callbacks):
        self._reset_callbacks.extend(callbacks)

    def on_reset(self):
        for cb in self._reset_callbacks:
            cb()

    def commit(self):
        """Snapshot the state (the rollback point after a failure), then check for added/removed
        workers — every rank reaches the same verdict, so all raise together."""
        self.save()
        self.commits += 1
        self.check_host_updates()

    def check_host_updates(self):
        ctx = basics._ctx
        if getattr(ctx, "elastic_gen", None) is None or ctx.store is None:
            return
        newer = 1 if current_generation(ctx.store) > ctx.elastic_gen else 0
        if basics.size() > 1:
            t = torch.tensor([newer], dtype=torch.int32, device=basics.device())
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            newer = int(t.item())
        if newer:
            raise HostsUpdatedInterrupt(skip_sync=False)

    def save(self):
        raise NotImplementedError

    def restore(self):
        raise NotImplementedError

    def sync(self):
        raise NotImplementedError


class ObjectState(State):
    """Plain Python attributes (epoch, batch, ...), broadcast from rank 0 on sync."""

    def __init__(self, **kwargs):
        super().__init__()
        self._keys = list(kwargs)
        for k, v in kwargs.items():
            setattr(self, k, v)
        self._saved = {}
        self.save()

    def save(self):
        self._saved = {k: copy.deepcopy(getattr(self, k)) for k in self._keys}

    def restore(self):
        for k, v in self._saved.items():
            setattr(self, k, copy.deepcopy(v))

    def sync(self):
        if basics.size() > 1:
            from .parallel.collectives import broadcast_object

            vals = broadcast_object({k: getattr(self, k) for k in self._keys}, root_rank=0)
            for k, v in vals.items():
                setattr(self, k, v)
        self.save()


class TorchState(ObjectState):
    """A torch model + optimizer (+ plain attributes): snapshots are host copies of the state
    dicts; ``sync`` broadcasts parameters and optimizer state from rank 0."""

    def __init__(self, model: torch.nn.Module | None = None, optimizer: torch.optim.Optimizer | None = None,
                 **kwargs):
        self.model = model
        self.optimizer = optimizer
        self._model_snap = None
        self._opt_snap = None
        super().__init__(**kwargs)

    def save(self):
        super().save()
        if self.model is not None:
            self._model_snap = {k: v.detach().to("cpu", copy=True) for k, v in self.model.state_dict().items()}
        if self.optimizer is not None:
            self._opt_snap = copy.deepcopy(_to_cpu(self.optimizer.state_dict()))

    def restore(self):
        super().restore()
        if self.model is not None and self._model_snap is not None:
            self.model.load_state_dict(self._model_snap)
        if self.optimizer is not None and self._opt_snap is not None:
            self.optimizer.load_state_dict(copy.deepcopy(self._opt_snap))

    def sync(self):
        from .parallel.optimizer import broadcast_optimizer_state, broadcast_parameters

        if hasattr(self.optimizer, "_elastic_reset"):
            self.optimizer._elastic_reset()
        if basics.size() > 1:
            if self.model is not None:
                broadcast_parameters(self.model.state_dict(), root_rank=0)
            if self.optimizer is not None:
                broadcast_optimizer_state(self.optimizer, root_rank=0)
        super().sync()


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


# ------------------------------------------------------------------------------------------ #
# run
# ------------------------------------------------------------------------------------------ #
def _membership_changed(grace_s: float) -> bool:
    """After a collective failure: did the driver publish a newer generation (a peer died)?"""
    ctx = basics._ctx
    if ctx.store is None or getattr(ctx, "elastic_gen", None) is None:
        return False
    deadline = time.time() + grace_s
    while time.time() < deadline:
        if current_generation(ctx.store) > ctx.elastic_gen:
            return True
        ctx.store.try_get(members_key(ctx.elastic_gen + 1), 0.5)
    return False


def _reset(failed: bool = False):
    """Re-form the world. ``failed``: after a collective failure, the old communicators are aborted
    instead of drained (a dead peer's bucket allreduce would never complete)."""
    basics.shutdown(abort=failed)
    basics.init()


def run(func):
    """Decorator: run ``func(state, ...)`` elastically (Horovod's ``hvd.elastic.run``)."""

    @functools.wraps(func)
    def wrapper(state: State, *args, **kwargs):
        if not basics.is_initialized():
            basics.init()
        grace = float(basics.config().elastic_grace_s)
        reset = failed = False
        while True:
            if reset:
                _reset(failed)
                state.on_reset()
                failed = False
            try:
                state.sync()
                return func(state, *args, **kwargs)
            except HostsUpdatedInterrupt as e:
                log.info("[rank %d] workers changed: re-forming the world", basics.rank())
                reset = True
                if not e.skip_sync:
                    state.save()
            except (HorovodInternalError, RuntimeError) as e:
                if not isinstance(e, HorovodInternalError) and not _membership_changed(grace):
                    raise
                log.warning("[rank %d] collective failed (%s): rolling back to the last commit", basics.rank(),
                            str(e).splitlines()[0][:200])
                state.restore()
                reset = failed = True

    return wrapper


__all__ = ["run", "State", "ObjectState", "TorchState", "HorovodInternalError", "HostsUpdatedInterrupt"]
