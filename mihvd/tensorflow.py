"""TF1-shaped training API: ``import mihvd.tensorflow as hvd``.

The reference's launched entrypoint (horovod/tensorflow_mnist.py) drives training with
``tf.train.MonitoredTrainingSession`` and three hooks (:138-150, :165-171). This module gives the
same control flow on PyTorch-ROCm:

* ``BroadcastGlobalVariablesHook(root_rank)`` — after the session is created *and* restored,
  broadcasts every global variable (weights, optimizer slots, global_step) from ``root_rank``.
* ``StopAtStepHook(last_step=...)``, ``LoggingTensorHook(tensors, every_n_iter)``,
  ``StepCounterHook`` (``global_step/sec``), ``CheckpointSaverHook`` (rank-0 ``./checkpoints``).
* ``MonitoredTrainingSession(checkpoint_dir, hooks, state=...)`` — restore latest checkpoint →
  hooks' ``after_create_session`` → ``run()`` loop with ``before_run``/``after_run`` → final save.

A *train state* object owns the variables (see ``TorchTrainState`` and
``mihvd.models.fused_mnist.FusedMNISTTrainer``): ``variables()`` maps TF names to tensors,
``load_variables()`` restores them, ``broadcast(root)`` syncs them, ``global_step`` counts steps.
"""
from __future__ import annotations

import logging
import time

import torch

from .basics import *  # noqa: F401,F403  (init, rank, size, Average, Adasum, ...)
from . import basics as _b
from .parallel.collectives import (allgather, allreduce, alltoall, barrier, broadcast, broadcast_,  # noqa: F401
                                   broadcast_object, grouped_allgather, grouped_allreduce, join, reducescatter)
from .parallel.compression import Compression  # noqa: F401
from .parallel.optimizer import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters  # noqa: F401
from .utils import checkpoint as ckpt
from .utils.logging import log_kv

log = logging.getLogger("mihvd")


# ------------------------------------------------------------------------------------------ #
# Train state
# ------------------------------------------------------------------------------------------ #
class TorchTrainState:
    """Variables of a TF-named torch model (``ordered_parameters()``) plus a torch Adam."""

    def __init__(self, model, optimizer=None):
        self.model = model
        self.optimizer = optimizer
        self.global_step = 0

    def named_variables(self):
        if hasattr(self.model, "ordered_parameters"):
            return list(self.model.ordered_parameters())
        return [(n.replace(".", "/"), p) for n, p in self.model.named_parameters()]

    def variables(self):
        return ckpt.adam_to_tf_vars(self.named_variables(), self.optimizer, self.global_step)

    def load_variables(self, variables):
        self.global_step = ckpt.tf_vars_to_adam(variables, self.named_variables(), self.optimizer)

    def broadcast(self, root_rank=0):
        broadcast_parameters(self.model.state_dict(), root_rank)
        if self.optimizer is not None:
            broadcast_optimizer_state(self.optimizer, root_rank)
        self.global_step = int(broadcast_object(self.global_step, root_rank))


# ------------------------------------------------------------------------------------------ #
# Hooks
# ------------------------------------------------------------------------------------------ #
class SessionRunArgs:
    def __init__(self, fetches=None):
        self.fetches = fetches


class SessionRunValues:
    def __init__(self, results):
        self.results = results


class SessionRunContext:
    def __init__(self, session):
        self.session = session
        self._stop = False
        self.steps = 1  # training steps this run advanced (a graph-replayed run covers several)

    def request_stop(self):
        self._stop = True
        self.session._stop_requested = True

    @property
    def stop_requested(self):
        return self._stop


class SessionRunHook:
    def begin(self):
        pass

    def after_create_session(self, session, coord=None):
        pass

    def before_run(self, run_context):
        return None

    def after_run(self, run_context, run_values):
        pass

    def end(self, session):
        pass


def broadcast_variables(variables, root_rank: int):
    """Broadcast tensors in place from ``root_rank`` (``hvd.broadcast_variables``): a mapping of
    name -> tensor (every rank must pass the same names) or a sequence of tensors."""
    items = sorted(variables.items()) if isinstance(variables, dict) else list(enumerate(variables))
    for name, t in items:
        broadcast_(t, root_rank, name=f"bcast.{name}")


def broadcast_global_variables(root_rank: int, state=None):
    """``hvd.broadcast_global_variables``: every global variable of a train state (weights, Adam
    slots, global_step; ``TorchTrainState`` / ``FusedMNISTTrainer``) from ``root_rank``."""
    if state is None:
        raise ValueError("broadcast_global_variables needs the train state whose variables to broadcast")
    state.broadcast(root_rank)


class BroadcastGlobalVariablesHook(SessionRunHook):
    """Broadcast all global variables from ``root_rank`` after session creation/restore
    (reference: horovod/tensorflow_mnist.py:139-143)."""

    def __init__(self, root_rank: int = 0, device: str = ""):
        self.root_rank = root_rank
        self.broadcasted = False

    def after_create_session(self, session, coord=None):
        session.state.broadcast(self.root_rank)
        self.broadcasted = True


class StopAtStepHook(SessionRunHook):
    def __init__(self, num_steps: int | None = None, last_step: int | None = None):
        if (num_steps is None) == (last_step is None):
            raise ValueError("exactly one of num_steps and last_step must be specified")
        self._num_steps = num_steps
        self._last_step = last_step

    def after_create_session(self, session, coord=None):
        if self._last_step is None:
            self._last_step = session.state.global_step + self._num_steps
        if session.state.global_step >= self._last_step:
            session._stop_requested = True

    def after_run(self, run_context, run_values):
        if run_context.session.state.global_step >= self._last_step:
            run_context.request_stop()

    @property
    def last_step(self):
        return self._last_step


class LoggingTensorHook(SessionRunHook):
    """Print named values every ``every_n_iter`` runs, on every rank (tensorflow_mnist.py:148-149).

    ``tensors`` maps display names to result keys (``'global_step'`` is the session's step)."""

    def __init__(self, tensors, every_n_iter: int = 10, formatter=None):
        if isinstance(tensors, (list, tuple)):
            tensors = {t: t for t in tensors}
        self.tensors = {k: (v if isinstance(v, str) else k) for k, v in tensors.items()}
        self.every_n = every_n_iter
        self.formatter = formatter
        self._iter = 0
        self._t = None
        self.lines: list[str] = []

    def after_run(self, run_context, run_values):
        # iteration cadence counted in training steps: a run that advanced k steps covers the
        # iterations [_iter, _iter + k); log if one of them is a multiple of every_n (k = 1: TF's rule)
        k = max(1, int(getattr(run_context, "steps", 1)))
        due = (self._iter + k - 1) // self.every_n * self.every_n >= self._iter
        if due:
            vals = {}
            res = run_values.results or {}
            for name, key in self.tensors.items():
                if key in ("global_step", "step") and key not in res:
                    v = run_context.session.state.global_step
                else:
                    v = res.get(key)
                if torch.is_tensor(v):
                    v = v.item() if v.numel() == 1 else v.tolist()
                vals[name] = v
            now = time.time()
            el = None if self._t is None else now - self._t
            self._t = now
            if self.formatter:
                line = self.formatter(vals)
                print(line, flush=True)
            else:
                line = log_kv("", **vals, **({"sec": round(el, 3)} if el is not None else {}))
            self.lines.append(line)
        self._iter += k


class StepCounterHook(SessionRunHook):
    """``global_step/sec`` (+ images/sec when ``batch_size`` is given) every N steps."""

    def __init__(self, every_n_steps: int = 100, batch_size: int | None = None, world_size: int | None = None):
        self.every_n = every_n_steps
        self.batch_size = batch_size
        self.world_size = world_size
        self._t0 = None
        self._s0 = None
        self.last_rate = None

    def after_create_session(self, session, coord=None):
        self._t0 = time.perf_counter()
        self._s0 = session.state.global_step

    def after_run(self, run_context, run_values):
        s = run_context.session.state.global_step
        if s - self._s0 >= self.every_n:
            session = run_context.session
            session.state_sync()
            now = time.perf_counter()
            rate = (s - self._s0) / (now - self._t0)
            self.last_rate = rate
            kv = {"global_step/sec": round(rate, 2)}
            if self.batch_size:
                ws = self.world_size or (_b.size() if _b.is_initialized() else 1)
                kv["img_per_sec"] = round(rate * self.batch_size * ws, 1)
            log_kv("", **kv)
            self._t0, self._s0 = now, s


class CheckpointSaverHook(SessionRunHook):
    """Rank-0 checkpoints in the TF1 layout (``checkpoint`` index + ``model.ckpt-<step>``).

    ``collective=True`` (a train state whose variables are sharded across ranks, e.g. the fused
    trainer's sharded dense/kernel optimizer): the hook runs on EVERY rank, all ranks call the
    state's collective ``gather_full_state()`` at the same step, and only the rank with a
    ``checkpoint_dir`` (rank 0) writes. Step triggers are deterministic on every rank; the time
    trigger is rank 0's clock, broadcast to the others every ``sync_steps`` steps."""

    def __init__(self, checkpoint_dir, save_secs=600, save_steps=None, max_to_keep=5, collective=False,
                 sync_steps=500):
        self.mgr = ckpt.CheckpointManager(checkpoint_dir, save_secs, save_steps, max_to_keep)
        self.writer = checkpoint_dir is not None
        self.collective = collective
        self.sync_steps = max(1, int(sync_steps))
        self.saved: list[str] = []
        self._prev = 0

    def after_create_session(self, session, coord=None):
        self.mgr._last_step = session.state.global_step
        self._prev = session.state.global_step

    def _due(self, step: int) -> bool:
        if not self.collective:
            return self.mgr.should_save(step)
        m = self.mgr
        due = bool(m.save_steps) and (m._last_step is None or step - m._last_step >= m.save_steps)
        if m.save_secs and step // self.sync_steps != self._prev // self.sync_steps:
            mine = (time.time() - m._last_t >= m.save_secs) if self.writer else None
            due = due or bool(broadcast_object(mine, 0))
        return due

    def _save(self, session, step: int):
        if self.collective and hasattr(session.state, "gather_full_state"):
            session.state.gather_full_state()  # collective: every rank, same step
        if self.writer:
            session.state_sync()
            self.saved.append(self.mgr.save(session.state.variables(), step))
        else:
            self.mgr._last_step, self.mgr._last_t = step, time.time()

    def after_run(self, run_context, run_values):
        step = run_context.session.state.global_step
        if self._due(step):
            self._save(run_context.session, step)
        self._prev = step

    def end(self, session):
        step = session.state.global_step
        if self.mgr._last_step != step:
            self._save(session, step)


# ------------------------------------------------------------------------------------------ #
# Session
# ------------------------------------------------------------------------------------------ #
class MonitoredTrainingSession:
    """Context manager mirroring ``tf.train.MonitoredTrainingSession`` semantics.

    ``run(train_op, feed_dict)`` calls ``train_op(**feed_dict)`` (or ``train_op(*feed_dict)``),
    increments ``global_step`` and returns the step's results dict."""

    def __init__(self, checkpoint_dir=None, hooks=(), config=None, state=None, save_checkpoint_secs=600,
                 save_checkpoint_steps=None, log_step_count_steps=None, max_to_keep=5, chief_only_hooks=()):
        if state is None:
            raise ValueError("MonitoredTrainingSession needs a train state (model variables)")
        self.state = state
        self.checkpoint_dir = checkpoint_dir
        self.hooks = list(hooks)
        # a state sharded across ranks checkpoints collectively: the saver hook runs on every rank
        collective = (hasattr(state, "gather_full_state") and _b.is_initialized() and _b.size() > 1)
        if (checkpoint_dir or collective) and (save_checkpoint_secs or save_checkpoint_steps):
            self.hooks.append(CheckpointSaverHook(checkpoint_dir, save_checkpoint_secs, save_checkpoint_steps, max_to_keep,
                                                  collective=collective))
        if log_step_count_steps:
            self.hooks.append(StepCounterHook(log_step_count_steps))
        self.hooks.extend(chief_only_hooks)
        self._stop_requested = False
        self.restored_from = None

    def state_sync(self):
        if hasattr(self.state, "sync"):
            self.state.sync()

    def __enter__(self):
        for h in self.hooks:
            h.begin()
        if self.checkpoint_dir:
            prefix = ckpt.latest_checkpoint(self.checkpoint_dir)
            if prefix is not None:
                self.state.load_variables(ckpt.Saver.restore(prefix))
                self.restored_from = prefix
                log.info("restored %s (global_step=%d)", prefix, self.state.global_step)
        for h in self.hooks:
            h.after_create_session(self, None)
        return self

    def should_stop(self) -> bool:
        return self._stop_requested

    def run(self, train_op, feed_dict=None):
        ctx = SessionRunContext(self)
        for h in self.hooks:
            h.before_run(ctx)
        before = self.state.global_step
        if feed_dict is None:
            res = train_op()
        elif isinstance(feed_dict, dict):
            res = train_op(**feed_dict)
        else:
            res = train_op(*feed_dict)
        if self.state.global_step == before:
            # states that count their own steps (the fused trainer) are not advanced twice
            self.state.global_step += 1
        ctx.steps = self.state.global_step - before
        if res is not None and not isinstance(res, dict):
            res = {"result": res}
        vals = SessionRunValues(res)
        for h in self.hooks:
            h.after_run(ctx, vals)
        return res

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None:
            for h in self.hooks:
                h.end(self)
        return False

    def close(self):
        self.__exit__(None, None, None)


from . import elastic  # noqa: E402,F401  (hvd.elastic)
