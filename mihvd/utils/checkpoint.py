"""Checkpoints in the reference's layout.

TF1 layout (horovod/tensorflow_mnist.py:157-167, MonitoredTrainingSession + Saver):
``<dir>/checkpoint`` (text index, ``model_checkpoint_path`` / ``all_model_checkpoint_paths``)
and ``<dir>/model.ckpt-<global_step>.pt`` holding every "global variable" by its TF name:
model variables, Adam slots ``<var>/Adam`` and ``<var>/Adam_1``, ``beta1_power``, ``beta2_power``
and ``global_step``. The newest ``max_to_keep`` (default 5) are kept. Writes are atomic
(temp file + ``os.replace``) and happen on rank 0 only; restore is followed by a broadcast.

Files are plain ``torch.save`` dicts of tensors, loadable with ``weights_only=True``.
"""
from __future__ import annotations

import os
import re
import tempfile
import time

import torch

INDEX = "checkpoint"
_PREFIX = "model.ckpt"


def _atomic_write_bytes(path: str, writer):
    d = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp-", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            writer(f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def read_index(ckpt_dir: str) -> tuple[str | None, list[str]]:
    p = os.path.join(ckpt_dir, INDEX)
    if not os.path.exists(p):
        return None, []
    latest, allp = None, []
    with open(p) as f:
        for line in f:
            m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths)\s*:\s*"(.*)"', line)
            if not m:
                continue
            if m.group(1) == "model_checkpoint_path":
                latest = m.group(2)
            else:
                allp.append(m.group(2))
    return latest, allp


def write_index(ckpt_dir: str, latest: str, all_paths: list[str]):
    text = f'model_checkpoint_path: "{latest}"\n' + "".join(f'all_model_checkpoint_paths: "{p}"\n' for p in all_paths)
    _atomic_write_bytes(os.path.join(ckpt_dir, INDEX), lambda f: f.write(text.encode()))


def latest_checkpoint(ckpt_dir: str) -> str | None:
    latest, _ = read_index(ckpt_dir)
    if latest is None:
        return None
    path = latest if os.path.isabs(latest) else os.path.join(ckpt_dir, latest)
    if os.path.exists(path + ".pt"):
        return path
    return None


class Saver:
    """``tf.train.Saver``-like: save(dict_of_tensors, global_step) -> prefix path."""

    def __init__(self, max_to_keep: int = 5):
        self.max_to_keep = max_to_keep

    def save(self, ckpt_dir: str, variables: dict[str, torch.Tensor], global_step: int) -> str:
        name = f"{_PREFIX}-{int(global_step)}"
        path = os.path.join(ckpt_dir, name)
        cpu = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else torch.tensor(v)) for k, v in variables.items()}
        _atomic_write_bytes(path + ".pt", lambda f: torch.save(cpu, f))
        _, allp = read_index(ckpt_dir)
        allp = [p for p in allp if p != name] + [name]
        while self.max_to_keep and len(allp) > self.max_to_keep:
            old = allp.pop(0)
            try:
                os.unlink(os.path.join(ckpt_dir, old + ".pt"))
            except FileNotFoundError:
                pass
        write_index(ckpt_dir, name, allp)
        return path

    @staticmethod
    def restore(prefix: str, map_location="cpu") -> dict[str, torch.Tensor]:
        return torch.load(prefix + ".pt", map_location=map_location, weights_only=True)


# ------------------------------------------------------------------------------------------ #
# Mapping a (TF-named) model + torch Adam into TF1 "global variables" and back.
# ------------------------------------------------------------------------------------------ #
def adam_to_tf_vars(named_params: list[tuple[str, torch.Tensor]], optimizer, global_step: int,
                    betas=(0.9, 0.999)) -> dict[str, torch.Tensor]:
    out: dict[str, torch.Tensor] = {}
    step = None
    for name, p in named_params:
        out[name] = p.detach()
        st = optimizer.state.get(p, {}) if optimizer is not None else {}
        if "exp_avg" in st:
            out[name + "/Adam"] = st["exp_avg"].detach()
            out[name + "/Adam_1"] = st["exp_avg_sq"].detach()
            step = st.get("step", step)
    if optimizer is not None:
        b1, b2 = optimizer.param_groups[0].get("betas", betas)
        t = float(step) if step is not None else 0.0
        out["beta1_power"] = torch.tensor(b1 ** (t + 1), dtype=torch.float32)
        out["beta2_power"] = torch.tensor(b2 ** (t + 1), dtype=torch.float32)
    out["global_step"] = torch.tensor(int(global_step), dtype=torch.int64)
    return out


def tf_vars_to_adam(variables: dict[str, torch.Tensor], named_params: list[tuple[str, torch.Tensor]], optimizer) -> int:
    """Load TF-named variables into params/Adam state. Returns the restored global_step."""
    b1 = optimizer.param_groups[0].get("betas", (0.9, 0.999))[0] if optimizer is not None else 0.9
    step = None
    if "beta1_power" in variables:
        bp = float(variables["beta1_power"])
        if 0 < bp < 1:
            import math

            step = round(math.log(bp) / math.log(b1)) - 1
    for name, p in named_params:
        with torch.no_grad():
            p.copy_(variables[name].to(p.device, p.dtype))
        if optimizer is not None and name + "/Adam" in variables:
            st = optimizer.state[p]
            st["exp_avg"] = variables[name + "/Adam"].to(p.device, p.dtype).clone()
            st["exp_avg_sq"] = variables[name + "/Adam_1"].to(p.device, p.dtype).clone()
            st["step"] = torch.tensor(float(step if step is not None else int(variables["global_step"])))
    return int(variables.get("global_step", torch.tensor(0)))


class CheckpointManager:
    """Time/step-triggered saving (TF ``CheckpointSaverHook`` defaults: every 600 s)."""

    def __init__(self, ckpt_dir: str, save_secs: float | None = 600, save_steps: int | None = None,
                 max_to_keep: int = 5):
        self.dir = ckpt_dir
        self.save_secs = save_secs
        self.save_steps = save_steps
        self.saver = Saver(max_to_keep)
        self._last_t = time.time()
        self._last_step = None

    def should_save(self, step: int) -> bool:
        if self.save_steps and (self._last_step is None or step - self._last_step >= self.save_steps):
            return True
        if self.save_secs and time.time() - self._last_t >= self.save_secs:
            return True
        return False

    def save(self, variables, step: int) -> str:
        self._last_t = time.time()
        self._last_step = step
        return self.saver.save(self.dir, variables, step)
