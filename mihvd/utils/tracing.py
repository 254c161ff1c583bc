"""roctx ranges for rocprofv3 ("roctx ranges around each kernel family").

``MIHVD_ROCTX=1`` makes :func:`trace_range` push/pop a roctx range (``torch.cuda.nvtx`` is backed by
roctx on ROCm builds of PyTorch), so ``rocprofv3 --marker-trace --kernel-trace`` shows the DP
engine's phases (bucket allreduces, synchronize, optimizer steps, fused training steps) next to the
kernels they launched. Off by default: a range costs a few microseconds of host time.
"""
from __future__ import annotations

import contextlib
import functools

import torch


@functools.lru_cache(maxsize=1)
def _enabled() -> bool:
    from .. import basics

    try:
        on = basics.config().roctx
    except Exception:
        import os

        on = os.environ.get("MIHVD_ROCTX", "0") in ("1", "true", "yes", "on")
    return bool(on) and torch.cuda.is_available()


def reset_cache():
    _enabled.cache_clear()


@contextlib.contextmanager
def trace_range(name: str):
    if not _enabled():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def mark(name: str):
    if _enabled():
        torch.cuda.nvtx.mark(name)
