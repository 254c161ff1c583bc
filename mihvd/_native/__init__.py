"""Loaders for the in-tree native libraries.

``runtime()`` returns the pybind11 host-runtime module, building it on first use if the ``.so``
is missing (it is git-ignored). ``load_kernels()`` loads ``libmihvd_kernels.so`` into
``torch.ops.mihvd``; on a machine with a GPU a missing or unloadable kernel library is an error
(no silent eager fallback), on a CPU-only machine it is reported as unavailable.
"""
from __future__ import annotations

import importlib
import os
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
_lock = threading.Lock()
_runtime = None
_kernels_loaded = None
_kernels_error = None


def runtime():
    global _runtime
    if _runtime is not None:
        return _runtime
    with _lock:
        if _runtime is None:
            from .. import _build

            if os.environ.get("MIHVD_NO_AUTOBUILD") != "1":
                _build.build_runtime()
            if _HERE not in sys.path:
                sys.path.insert(0, _HERE)
            _runtime = importlib.import_module("_mihvd_runtime")
    return _runtime


def kernels_path() -> str:
    return os.path.join(_HERE, "libmihvd_kernels.so")


def load_kernels(build_if_missing: bool = True) -> bool:
    """Load the HIP kernel library. Returns True when ``torch.ops.mihvd`` is populated."""
    global _kernels_loaded, _kernels_error
    if _kernels_loaded is not None:
        return _kernels_loaded
    with _lock:
        if _kernels_loaded is not None:
            return _kernels_loaded
        import torch

        path = kernels_path()
        try:
            if build_if_missing and os.environ.get("MIHVD_NO_AUTOBUILD") != "1":
                from .. import _build

                _build.build_kernels()
            torch.ops.load_library(path)
            _kernels_loaded = True
        except Exception as e:  # pragma: no cover - exercised only when the build is broken
            _kernels_error = e
            _kernels_loaded = False
    return _kernels_loaded


def kernels_error():
    return _kernels_error


def require_kernels():
    """Raise loudly if the HIP kernels are not loadable (used on GPU code paths)."""
    if not load_kernels():
        raise RuntimeError(
            "mihvd HIP kernel library %s could not be loaded: %r. Build it with "
            "`python -m mihvd._build kernels` (hipcc --offload-arch=gfx950)." % (kernels_path(), _kernels_error)
        )
