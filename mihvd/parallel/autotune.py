"""Fusion-threshold autotuner (Horovod ``HOROVOD_AUTOTUNE``).

Horovod's parameter manager runs a Bayesian search over fusion threshold and cycle time. mihvd has
no polling cycle (buckets are released by the in-order controller the moment they are complete), so
the one knob that matters is the bucket size: a grid search over ``MIHVD_AUTOTUNE_CANDIDATES``
(MiB). Each candidate runs ``trial_steps`` synchronized steps after ``warmup_steps``; the per-rank
median step times are max-reduced across ranks so every rank picks the same threshold, then the
optimizer re-plans its buckets once and tuning stops.
"""
from __future__ import annotations

import statistics
import time

import torch

from .. import basics
from ..utils.logging import log_kv


class FusionAutotuner:
    def __init__(self, candidates_mib, warmup_steps: int = 3, trial_steps: int = 8, log_file: str | None = None):
        self.candidates = [int(float(c) * 1024 * 1024) for c in candidates_mib]
        if not self.candidates:
            raise ValueError("autotune: no candidates")
        self.warmup = int(warmup_steps)
        self.trials = max(1, int(trial_steps))
        self.times: list[list[float]] = [[] for _ in self.candidates]
        self.idx = 0
        self.steps = 0
        self.done = False
        self.best: int | None = None
        self._t = None
        self.log_file = log_file or None  # horovodrun --autotune-log-file: one CSV row per candidate

    @classmethod
    def from_config(cls, cfg):
        return cls(cfg.autotune_candidates.split(","), cfg.autotune_warmup_steps, cfg.autotune_trial_steps,
                   getattr(cfg, "autotune_log", "") or None)

    def first(self) -> int:
        return self.candidates[0]

    def _now(self):
        if torch.cuda.is_available() and basics.device().type == "cuda":
            torch.cuda.synchronize(basics.device())
        return time.perf_counter()

    def on_step(self) -> int | None:
        """Call once per optimizer step (all ranks). Returns a new threshold to re-plan with, or None."""
        if self.done:
            return None
        now = self._now()
        prev, self._t = self._t, now
        self.steps += 1
        if prev is None or self.steps <= self.warmup + 1:
            return None
        self.times[self.idx].append(now - prev)
        if len(self.times[self.idx]) < self.trials:
            return None
        if self.idx + 1 < len(self.candidates):
            self.idx += 1
            self._t = None  # the re-plan step itself is not timed
            self.steps = self.warmup  # one warm step under the new plan
            return self.candidates[self.idx]
        return self._decide()

    def _decide(self) -> int:
        med = torch.tensor([statistics.median(t) for t in self.times], dtype=torch.float64)
        if basics.size() > 1:
            from .collectives import allreduce

            med = allreduce(med.to(basics.device()), op=basics.ReduceOp.Max, name="autotune").cpu()
        k = int(torch.argmin(med))
        self.best = self.candidates[k]
        self.done = True
        if basics.rank() == 0:
            log_kv("autotune", fusion_threshold_mib=round(self.best / 2 ** 20, 3),
                   **{f"ms@{c / 2 ** 20:g}MiB": round(float(m) * 1e3, 3) for c, m in zip(self.candidates, med)})
            if self.log_file:
                import csv
                import os

                new = not os.path.exists(self.log_file)
                with open(self.log_file, "a", newline="") as f:
                    w = csv.writer(f)
                    if new:
                        w.writerow(["fusion_threshold_bytes", "median_step_ms", "trial_steps", "chosen"])
                    for c, m in zip(self.candidates, med):
                        w.writerow([c, round(float(m) * 1e3, 4), self.trials, int(c == self.best)])
        return self.best
