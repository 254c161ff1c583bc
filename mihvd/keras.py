"""Keras-shaped training API: ``import mihvd.keras as hvd`` (horovod.tensorflow.keras parity).

The reference's GPU entrypoint (horovod/tensorflow_mnist_gpu.py) compiles a Keras model with a
Horovod-wrapped Adam and trains it with ``model.fit`` and two Horovod callbacks (:147-163):

* ``callbacks.BroadcastGlobalVariablesCallback(0)`` — broadcast model + optimizer variables at
  the end of the first batch (optimizer slots exist only after one step);
* ``callbacks.MetricAverageCallback()`` — allreduce-average the epoch metrics;
* rank 0 only: ``TensorBoard(log_dir='./logs')`` and ``ModelCheckpoint('./checkpoints/
  mnist-{epoch}.h5', save_best_only=True)``; at the end ``evaluate`` and ``save('./final_model')``.

``Model`` below provides ``compile / fit / evaluate / save`` over any torch module, with the
mixed-precision policy of the reference (:26-28) mapped to the MI355X-native ``bfloat16``
autocast (``'mixed_bfloat16'``, default) or ``'mixed_float16'`` with dynamic loss scaling.
"""
from __future__ import annotations

import math
import os
import sys
import time

import numpy as np
import torch

from .basics import *  # noqa: F401,F403
from . import basics as _b
from .parallel import collectives as C
from .parallel.compression import Compression  # noqa: F401
from .parallel.optimizer import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters  # noqa: F401
from .utils.logging import MetricsWriter


# ------------------------------------------------------------------------------------------ #
# Callbacks
# ------------------------------------------------------------------------------------------ #
class Callback:
    model: "Model" = None

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_batch_begin(self, batch, logs=None):
        pass

    def on_batch_end(self, batch, logs=None):
        pass


class BroadcastGlobalVariablesCallback(Callback):
    """``device``: Horovod's device for the broadcast ops (e.g. ``'/cpu:0'``). The variables are
    broadcast where they live (RCCL for device tensors, gloo for host tensors); a ``device`` naming
    the other kind is reported once, since moving ~39 MB of state through the host to honour it
    would only slow the broadcast down."""

    def __init__(self, root_rank: int = 0, device: str = ""):
        self.root_rank = root_rank
        self.device = device
        self.broadcast_done = False

    def set_model(self, model):
        super().set_model(model)
        want_cpu = "cpu" in str(self.device).lower()
        if self.device and model is not None and model.module is not None:
            on_cpu = next(model.module.parameters()).device.type == "cpu"
            if want_cpu != on_cpu:
                import warnings

                warnings.warn(f"BroadcastGlobalVariablesCallback(device={self.device!r}): the variables are "
                              f"broadcast on the device they live on ({'cpu' if on_cpu else 'gpu'})")

    def on_batch_end(self, batch, logs=None):
        if self.broadcast_done:
            return
        broadcast_parameters(self.model.module.state_dict(), self.root_rank)
        broadcast_optimizer_state(self.model.optimizer, self.root_rank)
        self.broadcast_done = True


class MetricAverageCallback(Callback):
    """Average every numeric entry of ``logs`` across ranks with one fused allreduce."""

    def __init__(self, device: str = ""):
        pass

    def on_epoch_end(self, epoch, logs=None):
        if logs is None or not _b.is_initialized() or _b.size() == 1:
            return
        keys = sorted(k for k, v in logs.items() if isinstance(v, (int, float, np.floating)))
        if not keys:
            return
        t = torch.tensor([float(logs[k]) for k in keys], dtype=torch.float64, device=_b.device())
        t = C.allreduce(t, op=_b.Average, name="metrics")
        for k, v in zip(keys, t.tolist()):
            logs[k] = v


class LearningRateWarmupCallback(Callback):
    """Linear LR warmup from ``initial_lr / size`` to ``initial_lr`` over ``warmup_epochs``."""

    def __init__(self, initial_lr, warmup_epochs=5, momentum_correction=True, steps_per_epoch=None, verbose=0):
        self.initial_lr = initial_lr
        self.warmup_epochs = warmup_epochs
        self.momentum_correction = momentum_correction
        self.steps_per_epoch = steps_per_epoch
        self.verbose = verbose
        self._epoch = 0
        self._restore_momentum = None

    def on_epoch_begin(self, epoch, logs=None):
        self._epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        if self._epoch >= self.warmup_epochs:
            return
        spe = self.steps_per_epoch or self.model._steps_per_epoch or 1
        progress = (self._epoch + batch / spe) / self.warmup_epochs
        size = _b.size() if _b.is_initialized() else 1
        lr = self.initial_lr / size * (1 + progress * (size - 1))
        _set_lr(self.model.optimizer, lr, self.momentum_correction, self)

    def on_batch_end(self, batch, logs=None):
        _restore_momentum(self.model.optimizer, self)

    def on_epoch_end(self, epoch, logs=None):
        if self.verbose and epoch == self.warmup_epochs - 1 and (not _b.is_initialized() or _b.rank() == 0):
            print(f"Epoch {epoch + 1}: finished gradual learning rate warmup to {self.initial_lr:g}.", flush=True)


def _set_lr(optimizer, lr, momentum_correction, owner):
    """Set every param group's LR. With ``momentum_correction`` (Horovod's rule, Goyal et al.
    2017), an optimizer with a momentum buffer (SGD's ``momentum``) scales its momentum by
    new_lr / old_lr for the batch the LR changes in, so the accumulated velocity is not applied at
    the new LR; the callback restores the momentum at the batch end. Adam has no such term."""
    saved = []
    for g in optimizer.param_groups:
        old = g["lr"]
        if momentum_correction and g.get("momentum") and old > 0 and lr != old:
            saved.append((g, g["momentum"]))
            g["momentum"] = g["momentum"] * lr / old
        g["lr"] = lr
    owner._restore_momentum = saved or None


def _restore_momentum(optimizer, owner):
    if owner._restore_momentum:
        for g, m in owner._restore_momentum:
            g["momentum"] = m
        owner._restore_momentum = None


class LearningRateScheduleCallback(Callback):
    """Horovod's ``LearningRateScheduleCallback``: between ``start_epoch`` and ``end_epoch`` the LR is
    ``initial_lr * multiplier(epoch)`` — per epoch (``staircase=True``) or per batch with a fractional
    epoch. ``multiplier`` may be a constant."""

    def __init__(self, initial_lr, multiplier, start_epoch=0, end_epoch=None, staircase=True,
                 momentum_correction=True, steps_per_epoch=None, verbose=0):
        self.momentum_correction = momentum_correction
        self._restore_momentum = None
        self.initial_lr = initial_lr
        self.multiplier = multiplier if callable(multiplier) else (lambda epoch, m=multiplier: m)
        self.start_epoch = start_epoch
        self.end_epoch = end_epoch
        self.staircase = staircase
        self.steps_per_epoch = steps_per_epoch
        self._epoch = 0

    def _active(self, epoch) -> bool:
        return epoch >= self.start_epoch and (self.end_epoch is None or epoch < self.end_epoch)

    def _set(self, lr):
        _set_lr(self.model.optimizer, lr, self.momentum_correction, self)

    def on_batch_end(self, batch, logs=None):
        _restore_momentum(self.model.optimizer, self)

    def on_epoch_begin(self, epoch, logs=None):
        self._epoch = epoch
        if self.staircase and self._active(epoch):
            self._set(self.initial_lr * self.multiplier(epoch))

    def on_batch_begin(self, batch, logs=None):
        if self.staircase or not self._active(self._epoch):
            return
        spe = self.steps_per_epoch or self.model._steps_per_epoch or 1
        self._set(self.initial_lr * self.multiplier(self._epoch + batch / spe))


class ModelCheckpoint(Callback):
    def __init__(self, filepath, monitor="val_loss", save_best_only=False, mode="min", verbose=0):
        self.filepath = filepath
        self.monitor = monitor
        self.save_best_only = save_best_only
        self.mode = mode
        self.best = math.inf if mode == "min" else -math.inf
        self.saved: list[str] = []

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        path = self.filepath.format(epoch=epoch + 1, **{k: v for k, v in logs.items()})
        cur = logs.get(self.monitor)
        if self.save_best_only:
            if cur is None:
                return
            better = cur < self.best if self.mode == "min" else cur > self.best
            if not better:
                return
            self.best = cur
        self.model.save(path)
        self.saved.append(path)


class TensorBoard(Callback):
    """Scalar logging to ``<log_dir>/metrics.jsonl`` (TensorBoard itself is not installed)."""

    def __init__(self, log_dir="./logs", **kw):
        self.log_dir = log_dir
        self.writer = None

    def on_train_begin(self, logs=None):
        self.writer = MetricsWriter(self.log_dir)

    def on_epoch_end(self, epoch, logs=None):
        if self.writer:
            self.writer.scalars({k: v for k, v in (logs or {}).items() if isinstance(v, (int, float))}, epoch)

    def on_train_end(self, logs=None):
        if self.writer:
            self.writer.close()


class _CallbacksNS:
    BroadcastGlobalVariablesCallback = BroadcastGlobalVariablesCallback
    MetricAverageCallback = MetricAverageCallback
    LearningRateWarmupCallback = LearningRateWarmupCallback
    LearningRateScheduleCallback = LearningRateScheduleCallback
    ModelCheckpoint = ModelCheckpoint
    TensorBoard = TensorBoard
    Callback = Callback


callbacks = _CallbacksNS()


# ------------------------------------------------------------------------------------------ #
# Model
# ------------------------------------------------------------------------------------------ #
class _LossScaler:
    """Dynamic loss scaling for the fp16 policy (Keras LossScaleOptimizer semantics: start at
    2**15, halve on overflow and skip the step, double after ``growth_interval`` clean steps).

    On a GPU the state is the device pair ``ls = [scale, found_nonfinite]`` driven by the HIP
    kernels ``grad_check_`` (multi-tensor unscale + non-finite test) and ``update_scale_``
    (csrc/kernels/dp_kernels.hip); the host reads one flag per step to decide
    whether to apply the update. On the CPU the same rule runs in plain torch."""

    def __init__(self, init_scale=2.0 ** 15, growth_interval=2000):
        self.init_scale = float(init_scale)
        self.growth_interval = growth_interval
        self.good_steps = 0
        self._scale = float(init_scale)
        self._ls = None
        self._tracker = None

    def _device_state(self, device):
        if device.type != "cuda":
            return None
        if self._ls is None:
            from . import _native

            _native.require_kernels()
            self._ls = torch.tensor([self._scale, 0.0], dtype=torch.float32, device=device)
            self._tracker = torch.zeros(1, dtype=torch.int32, device=device)
        return self._ls

    @property
    def scale(self):
        return self._ls[0] if self._ls is not None else self._scale

    def scale_loss(self, loss):
        ls = self._device_state(loss.device)
        return loss * (ls[0] if ls is not None else self._scale)

    def unscale_and_check(self, params) -> bool:
        grads = [p.grad for p in params if p.grad is not None]
        if not grads:
            return True
        ls = self._device_state(grads[0].device)
        if ls is not None:
            ops = torch.ops.mihvd
            ops.grad_check_([g for g in grads if g.dtype == torch.float32], ls, True)
            finite = float(ls[1].item()) == 0.0
            ops.update_scale_(ls, self._tracker, 2.0, 0.5, self.growth_interval, 1.0)
            return finite
        finite = True
        for g in grads:
            g.div_(self._scale)
            if not torch.isfinite(g).all():
                finite = False
        if finite:
            self.good_steps += 1
            if self.good_steps >= self.growth_interval:
                self._scale *= 2
                self.good_steps = 0
        else:
            self._scale = max(1.0, self._scale / 2)
            self.good_steps = 0
        return finite


class Model:
    """``policy`` is the Keras mixed-precision policy (tensorflow_mnist_gpu.py:26-28). A module with
    ``impl == "hip"`` (``MNISTConvNet(impl="hip")``) trains through the hand-written CDNA4 kernels:
    under ``float32`` / ``mixed_bfloat16`` / ``mixed_float16`` with a TF1/Keras-rule Adam, ``fit`` drives the fused,
    graph-replayed training step (``FusedMNISTTrainer``: the whole step in seven launches, k steps per
    HIP graph replay between callback points); otherwise one fused forward+backward autograd node
    per batch: ``float32`` runs the exact-fp32 kernels,
    ``mixed_bfloat16`` the bf16-operand kernels (fp32 accumulation and master weights),
    ``mixed_float16`` the same kernels built with fp16 operands (v_mfma_f32_16x16x32_f16) under the
    HIP dynamic loss scaler: the kernels scale dz by the current scale, the scaler unscales, checks
    for overflow and skips the step on inf/NaN (Keras LossScaleOptimizer semantics)."""

    def __init__(self, module: torch.nn.Module, policy: str = "float32"):
        self.module = module
        self.policy = policy
        if getattr(module, "impl", None) == "hip":
            module.hip_precision = {"float32": "fp32", "mixed_float16": "fp16"}.get(policy, "bf16")
        self.optimizer = None
        self.loss_fn = None
        self.metrics = []
        self.history = {}
        self._steps_per_epoch = None
        self._scaler = _LossScaler() if policy == "mixed_float16" else None

    def compile(self, optimizer, loss, metrics=()):
        self.optimizer = optimizer
        self.loss_fn = loss
        self.metrics = list(metrics)

    def _device(self):
        return next(self.module.parameters()).device

    def _autocast(self):
        dev = self._device().type
        if self.policy == "mixed_bfloat16":
            return torch.autocast(dev, dtype=torch.bfloat16)
        if self.policy == "mixed_float16":
            return torch.autocast(dev, dtype=torch.float16)
        return torch.autocast(dev, enabled=False)

    def _batch(self, x, y, idx):
        dev = self._device()
        xb = torch.as_tensor(x[idx], device=dev).float()
        yb = torch.as_tensor(y[idx], device=dev).long()
        return xb, yb

    def train_on_batch(self, xb, yb):
        self.module.train()
        self.optimizer.zero_grad()
        if getattr(self.module, "impl", None) == "hip":
            # whole forward+backward in the CDNA4 kernels, one autograd node (MFMA inside)
            from .ops.functional import fused_mnist_loss

            S = float(self._scaler.scale) if self._scaler is not None else None
            loss, acc = fused_mnist_loss(self.module, xb, yb, training=True, return_accuracy=True, loss_scale=S)
            if self._scaler is None:
                loss.backward()
                self.optimizer.step()
                return loss.detach(), acc
            logits = None
        else:
            with self._autocast():
                logits = self.module(xb)
            loss = self.loss_fn(logits.float(), yb)
        if self._scaler is not None:
            self._scaler.scale_loss(loss).backward()
            self.optimizer.synchronize()
            ok = self._scaler.unscale_and_check([p for g in self.optimizer.param_groups for p in g["params"]])
            if ok:
                with self.optimizer.skip_synchronize():
                    self.optimizer.step()
            else:
                self.optimizer._synchronized = False
        else:
            loss.backward()
            self.optimizer.step()
        if logits is not None:
            acc = (logits.argmax(1) == yb).float().mean()
        return loss.detach(), acc.detach()

    @torch.no_grad()
    def evaluate(self, x, y, batch_size=100, steps=None, verbose=0):
        self.module.eval()
        n = len(x)
        steps = steps or max(1, n // batch_size)
        tot_loss = torch.zeros((), device=self._device())
        tot_acc = torch.zeros((), device=self._device())
        for s in range(steps):
            idx = np.arange(s * batch_size, min(n, (s + 1) * batch_size))
            xb, yb = self._batch(x, y, idx)
            with self._autocast():
                logits = self.module(xb)
            tot_loss += self.loss_fn(logits.float(), yb)
            tot_acc += (logits.argmax(1) == yb).float().mean()
        return [float(tot_loss) / steps, float(tot_acc) / steps]

    # callbacks whose per-batch hooks the fused fit path reproduces (or that have none)
    _FUSED_CALLBACKS = (BroadcastGlobalVariablesCallback, MetricAverageCallback, ModelCheckpoint, TensorBoard)

    def _fused_fit_trainer(self, cbs, batch_size):
        """The graph-replayed fit path (tensorflow_mnist_gpu.py:166-182 under ``float32``,
        ``mixed_bfloat16`` or ``mixed_float16``, the last with the device loss scaler in the graph): a :class:`~mihvd.models.fused_mnist.FusedMNISTTrainer` over the
        module's weights and the optimizer's Adam hyper-parameters, or None where the per-batch path
        must run (MIHVD_KERAS_FUSED=0, another policy or module, an optimizer or reduction the fused
        step does not implement, existing optimizer state, or a callback with per-batch hooks)."""
        ok = self._fused_fit_eligible(cbs, batch_size)
        # Every rank must take the same path: building the trainer is collective and the two paths
        # issue different collectives. The reference idiom gives rank 0 extra callbacks
        # (tensorflow_mnist_gpu.py:156-163), so one rank's list can rule the fused path out: agree
        # on the minimum before choosing.
        if _b.is_initialized() and _b.size() > 1:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                                device=_b.device() if _b.backend() == "nccl" else "cpu")
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
            ok = bool(flag.item())
        if not ok:
            return None
        m, opt = self.module, self.optimizer
        g = opt.param_groups[0]
        op = getattr(opt, "_op", _b.Average)
        from .models.fused_mnist import FusedMNISTTrainer

        precision = {"float32": "fp32", "mixed_float16": "fp16"}.get(self.policy, "bf16")
        tr = FusedMNISTTrainer(batch_size=batch_size, lr=g["lr"], betas=tuple(g["betas"]), eps=g["eps"],
                               dropout=m.dropout_rate, device=self._device(), op=op, precision=precision)
        if precision == "fp16" and self._scaler is not None and self._scaler._ls is not None:
            tr.loss_scale.copy_(self._scaler._ls)  # continue from the per-batch path's scale
        tr.load_model_weights(m)
        tr.track_stats = True
        return tr

    def _fused_fit_eligible(self, cbs, batch_size) -> bool:
        """This rank's view of whether the fused fit path applies (see _fused_fit_trainer)."""
        if os.environ.get("MIHVD_KERAS_FUSED", "1") == "0":
            return False
        from .models.mnist import MNISTConvNet
        from .optim import FusedAdam, TFAdam

        m, opt = self.module, self.optimizer
        if (not isinstance(m, MNISTConvNet) or getattr(m, "impl", None) != "hip" or self.policy not in
                ("float32", "mixed_bfloat16", "mixed_float16") or opt is None or not 1 <= batch_size <= 128):
            return False
        if not isinstance(opt, (TFAdam, FusedAdam)) or len(opt.param_groups) != 1 or any(opt.state.values()):
            return False
        g = opt.param_groups[0]
        if isinstance(opt, FusedAdam) and (g.get("rule") != "tf" or g.get("weight_decay", 0.0) != 0.0):
            return False
        if getattr(opt, "_op", _b.Average) not in (_b.Average, _b.Sum):
            return False
        for cb in cbs:
            if not isinstance(cb, self._FUSED_CALLBACKS):
                overridden = (type(cb).on_batch_begin is not Callback.on_batch_begin
                              or type(cb).on_batch_end is not Callback.on_batch_end)
                if overridden:
                    return False
        return True

    def _fit_fused(self, tr, x, y, batch_size, epochs, steps_per_epoch, validation_data, validation_steps, cbs,
                   verbose, shuffle, seed):
        """fit() on the fused trainer: the dataset resident on the device, each epoch's steps replayed
        from HIP graphs of ``MIHVD_KERAS_GRAPH_STEPS`` steps (default 20) between the callback points
        (BroadcastGlobalVariablesCallback after the first batch, the epoch-end callbacks); the
        module's weights are synchronised at every epoch end (validation, checkpoints) and the
        optimizer's Adam slots at the end of fit."""
        k = int(os.environ.get("MIHVD_KERAS_GRAPH_STEPS", "20"))
        tr.set_device_dataset(torch.as_tensor(np.asarray(x, dtype=np.float32)),
                              torch.as_tensor(np.asarray(y).astype(np.int64)), shuffle=shuffle,
                              seed=0 if seed is None else int(seed))
        bcast = [cb for cb in cbs if isinstance(cb, BroadcastGlobalVariablesCallback)]
        self.fused_trainer = tr
        t_epochs = []
        for epoch in range(epochs):
            for cb in cbs:
                cb.on_epoch_begin(epoch)
            # an epoch-level callback (on_epoch_begin only: it passed the filter) may have changed the
            # LR; the trainer bakes it into its graphs, so a change re-captures them
            tr.set_lr(self.optimizer.param_groups[0]["lr"])
            t0 = time.time()
            tr.reset_stats()
            done = 0
            if epoch == 0:
                tr.device_step()  # batch 0 eagerly: the broadcast callback's point (optimizer state exists)
                done = 1
                for cb in bcast:
                    if not cb.broadcast_done:
                        tr.broadcast(cb.root_rank)
                        cb.broadcast_done = True
            tr.run_steps(steps_per_epoch - done, steps_per_replay=k)
            loss, acc = tr.epoch_stats()  # (synchronises)
            t_epochs.append(time.time() - t0)
            tr.sync()
            tr.gather_full_state()
            tr.to_model(self.module)
            logs = {"loss": loss, "accuracy": acc}
            if validation_data is not None:
                vl, va = self.evaluate(validation_data[0], validation_data[1], batch_size, validation_steps)
                logs["val_loss"], logs["val_accuracy"] = vl, va
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            for k2, v in logs.items():
                self.history.setdefault(k2, []).append(v)
            if verbose:
                dt = time.time() - t0
                print(f"Epoch {epoch + 1}/{epochs} - {dt:.1f}s - " +
                      " - ".join(f"{k2}: {v:.4f}" for k2, v in logs.items()), file=sys.stdout, flush=True)
        # the Adam slots into the optimizer's state (a later per-batch fit or a checkpoint continues
        # from them), and under mixed_float16 the device loss scale into the model's scaler
        self._adam_state_from_trainer(tr)
        if getattr(tr, "f16", False) and self._scaler is not None:
            self._scaler._device_state(tr.device)
            self._scaler._ls.copy_(tr.loss_scale)
        # images/sec of the training steps (whole job), from the epochs after the first (whose time
        # includes the HIP graph captures) when there are several
        per_epoch = steps_per_epoch * batch_size * (_b.size() if _b.is_initialized() else 1)
        timed = t_epochs[1:] if len(t_epochs) > 1 else t_epochs
        self.fit_throughput = per_epoch * len(timed) / sum(timed) if sum(timed) > 0 else float("nan")
        for cb in cbs:
            cb.on_train_end()
        return self

    def _adam_state_from_trainer(self, tr):
        opt = self.optimizer
        names = dict(self.module.ordered_parameters())
        t = int(tr.state[1].item())
        for name, p in names.items():
            st = opt.state[p]
            st["step"] = torch.tensor(float(t))
            st["exp_avg"] = tr.pview(name, tr.m).detach().clone().view_as(p)
            st["exp_avg_sq"] = tr.pview(name, tr.v).detach().clone().view_as(p)

    def fit(self, x, y, batch_size=100, epochs=1, steps_per_epoch=None, validation_data=None, validation_steps=None,
            callbacks=(), verbose=1, shuffle=True, seed=None):
        cbs = list(callbacks)
        for cb in cbs:
            cb.set_model(self)
        n = len(x)
        tr = self._fused_fit_trainer(cbs, batch_size)
        if tr is not None:
            steps_per_epoch = steps_per_epoch or max(1, n // batch_size)
            self._steps_per_epoch = steps_per_epoch
            for cb in cbs:
                cb.on_train_begin()
            try:
                return self._fit_fused(tr, x, y, batch_size, epochs, steps_per_epoch, validation_data,
                                       validation_steps, cbs, verbose, shuffle, seed)
            finally:
                tr.close()
        steps_per_epoch = steps_per_epoch or max(1, n // batch_size)
        self._steps_per_epoch = steps_per_epoch
        rng = np.random.default_rng(seed)
        for cb in cbs:
            cb.on_train_begin()
        perm = rng.permutation(n) if shuffle else np.arange(n)
        pos = 0
        for epoch in range(epochs):
            for cb in cbs:
                cb.on_epoch_begin(epoch)
            t0 = time.time()
            sum_loss = torch.zeros((), device=self._device())
            sum_acc = torch.zeros((), device=self._device())
            for step in range(steps_per_epoch):
                if pos + batch_size > n:
                    perm = rng.permutation(n) if shuffle else np.arange(n)
                    pos = 0
                idx = perm[pos:pos + batch_size]
                pos += batch_size
                for cb in cbs:
                    cb.on_batch_begin(step)
                xb, yb = self._batch(x, y, idx)
                loss, acc = self.train_on_batch(xb, yb)
                sum_loss += loss
                sum_acc += acc
                for cb in cbs:
                    cb.on_batch_end(step, {})
            logs = {"loss": float(sum_loss) / steps_per_epoch, "accuracy": float(sum_acc) / steps_per_epoch}
            if validation_data is not None:
                vl, va = self.evaluate(validation_data[0], validation_data[1], batch_size, validation_steps)
                logs["val_loss"], logs["val_accuracy"] = vl, va
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            for k, v in logs.items():
                self.history.setdefault(k, []).append(v)
            if verbose:
                dt = time.time() - t0
                print(f"Epoch {epoch + 1}/{epochs} - {dt:.1f}s - " +
                      " - ".join(f"{k}: {v:.4f}" for k, v in logs.items()), file=sys.stdout, flush=True)
        for cb in cbs:
            cb.on_train_end()
        return self

    def save(self, path: str):
        """Save weights + optimizer state. A path without an extension is treated as a
        directory (the SavedModel shape of ``model.save('./final_model')``)."""
        state = {"model": {k: v.detach().cpu() for k, v in self.module.state_dict().items()}}
        if os.path.splitext(path)[1] == "":
            os.makedirs(path, exist_ok=True)
            target = os.path.join(path, "model.pt")
        else:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            target = path
        tmp = target + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, target)
        return target

    @staticmethod
    def load_weights(module, path: str):
        target = os.path.join(path, "model.pt") if os.path.isdir(path) else path
        sd = torch.load(target, map_location="cpu", weights_only=True)["model"]
        module.load_state_dict(sd)
        return module


# ------------------------------------------------------------------------------------------ #
# Module-level functions of horovod.tensorflow.keras
# ------------------------------------------------------------------------------------------ #
def _as_tensor(value):
    t = value if torch.is_tensor(value) else torch.as_tensor(np.asarray(value))
    return t.to(_b.device()) if _b.is_initialized() and _b.backend() == "nccl" else t


def _like(value, t: torch.Tensor):
    """Return ``t`` in the caller's type: a tensor for a tensor, a numpy array otherwise (Keras
    backend values), a Python scalar for a scalar."""
    if torch.is_tensor(value):
        return t.to(value.device)
    a = t.detach().cpu().numpy()
    return a.item() if np.ndim(value) == 0 and a.size == 1 else a


def allreduce(value, name=None, average=True, prescale_factor=1.0, postscale_factor=1.0, op=None,
              compression=Compression.none):
    """``hvd.allreduce`` of a tensor / array / scalar (Average unless ``average=False`` or ``op``)."""
    t = _as_tensor(value)
    if not t.is_floating_point():
        t = t.double() if not torch.is_tensor(value) else t
    if op is None:
        op = _b.Average if average else _b.Sum
    return _like(value, C.allreduce(t, name=name, op=op, prescale_factor=prescale_factor,
                                    postscale_factor=postscale_factor, compression=compression))


def allgather(value, name=None):
    """``hvd.allgather``: concatenation of every rank's value along the first dimension."""
    return _like(value, C.allgather(_as_tensor(value), name=name))


def broadcast(value, root_rank, name=None):
    """``hvd.broadcast``: ``root_rank``'s value on every rank."""
    return _like(value, C.broadcast(_as_tensor(value), root_rank, name=name))


def broadcast_global_variables(root_rank: int, model: "Model"):
    """Broadcast a compiled model's weights and optimizer state from ``root_rank`` (Horovod's
    Keras form reads them from the global backend session; here the model is passed)."""
    broadcast_parameters(model.module.state_dict(), root_rank)
    if model.optimizer is not None:
        broadcast_optimizer_state(model.optimizer, root_rank)


def load_model(filepath: str, module: torch.nn.Module, optimizer=None, loss=None, metrics=(),
               compression=Compression.none, policy: str = "float32", custom_optimizers=None,
               custom_objects=None) -> "Model":
    """``hvd.load_model``: a ``Model`` over ``module`` with the weights saved by ``Model.save`` and,
    if ``optimizer`` is given (an optimizer over ``module``'s parameters, or a factory / optimizer
    class called with them; also taken from ``custom_optimizers``), that optimizer wrapped in
    ``DistributedOptimizer``. The architecture is passed as
    ``module``: a torch checkpoint holds tensors only (weights-only load)."""
    Model.load_weights(module, filepath)
    m = Model(module, policy=policy)
    if optimizer is None and custom_optimizers:
        optimizer = custom_optimizers[0] if isinstance(custom_optimizers, (list, tuple)) else custom_optimizers
    if optimizer is not None and not isinstance(optimizer, torch.optim.Optimizer):
        optimizer = optimizer(module.parameters())  # a factory / optimizer class over the parameters
    if optimizer is not None:
        optimizer = DistributedOptimizer(optimizer, named_parameters=module.named_parameters(), compression=compression)
    m.compile(optimizer, loss, metrics)
    return m


from . import elastic  # noqa: E402,F401  (hvd.elastic)
