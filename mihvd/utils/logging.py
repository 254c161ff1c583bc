"""Rank-prefixed, Promtail/Loki-friendly logging and a JSON-lines metrics writer.

Every line is ``[rank r/size] key=value ...`` so a LogQL query such as
``{namespace="ml-ops"} |= "img_per_sec" | logfmt`` can parse it. The reference's only signals are
``step``/``loss`` every 10 iterations on every rank (horovod/tensorflow_mnist.py:148-149) and TF's
``global_step/sec``; both are emitted in this format.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time


def _rank_size():
    try:
        from .. import basics

        if basics.is_initialized():
            return basics.rank(), basics.size()
    except Exception:
        pass
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def fmt_kv(**kv) -> str:
    parts = []
    for k, v in kv.items():
        if isinstance(v, float):
            parts.append(f"{k}={v:.6g}")
        else:
            parts.append(f"{k}={v}")
    return " ".join(parts)


def log_kv(msg: str = "", stream=None, **kv):
    r, n = _rank_size()
    line = f"[rank {r}/{n}] " + (msg + " " if msg else "") + fmt_kv(**kv)
    print(line, file=stream or sys.stdout, flush=True)
    return line


class MetricsWriter:
    """Append-only JSONL scalar log (a TensorBoard-equivalent for ``./logs``)."""

    def __init__(self, log_dir: str, filename: str = "metrics.jsonl"):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, filename)
        self._f = open(self.path, "a", buffering=1)
        self._lock = threading.Lock()

    def scalar(self, tag: str, value: float, step: int):
        rec = {"wall_time": time.time(), "step": int(step), "tag": tag, "value": float(value)}
        with self._lock:
            self._f.write(json.dumps(rec) + "\n")

    def scalars(self, values: dict, step: int):
        for k, v in values.items():
            self.scalar(k, v, step)

    def close(self):
        with self._lock:
            if not self._f.closed:
                self._f.close()
