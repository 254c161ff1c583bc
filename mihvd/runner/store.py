"""The native rendezvous store as a ``torch.distributed.Store``.

``mihvdrun`` hosts a :class:`StoreServer` (C++, ``csrc/runtime/store.cc``) — the equivalent of the
rendezvous server ``horovodrun`` starts — and exports its address as ``MIHVD_STORE_ADDR=host:port``.
``mihvd.init()`` then builds the process group on :class:`NativeStore`, so the RCCL unique-id
exchange, gloo's pairwise bootstrap and the negotiation engine (``mihvd/parallel/engine.py``) all
run over the framework's own control plane instead of torch's TCPStore.
"""
from __future__ import annotations

import datetime
import os

import torch.distributed as dist

from .._native import runtime

ENV_ADDR = "MIHVD_STORE_ADDR"


def parse_addr(addr: str) -> tuple[str, int]:
    host, port = addr.rsplit(":", 1)
    return host.strip("[]"), int(port)


def start_server(host: str = "0.0.0.0", port: int = 0):
    """Start a store server in this process (background thread); ``.port`` is the bound port."""
    return runtime().StoreServer(host, port)


class NativeStore(dist.Store):
    """``torch.distributed.Store`` backed by the C++ StoreClient (one TCP connection)."""

    def __init__(self, host: str, port: int, timeout: datetime.timedelta = datetime.timedelta(seconds=600),
                 connect_timeout_s: float = 120.0):
        super().__init__()
        self.host, self.port = host, int(port)
        self._client = runtime().StoreClient(host, int(port), float(connect_timeout_s))
        self._timeout_s = timeout.total_seconds()

    @classmethod
    def from_env(cls, timeout: datetime.timedelta = datetime.timedelta(seconds=600)) -> "NativeStore | None":
        addr = os.environ.get(ENV_ADDR)
        if not addr:
            return None
        h, p = parse_addr(addr)
        return cls(h, p, timeout)

    # torch.distributed.Store interface -------------------------------------------------------
    def set(self, key, value):
        self._client.set(key, _as_bytes(value))

    def get(self, key):
        return self._client.get(key, self._timeout_s)

    def add(self, key, value):
        return self._client.add(key, int(value))

    def compare_set(self, key, expected_value, desired_value):
        return self._client.compare_set(key, _as_bytes(expected_value), _as_bytes(desired_value))

    def check(self, keys):
        return self._client.check(list(keys))

    def wait(self, keys, timeout=None):
        t = self._timeout_s if timeout is None else (timeout.total_seconds() if hasattr(timeout, "total_seconds")
                                                      else float(timeout))
        if not self._client.wait(list(keys), t):
            raise RuntimeError(f"NativeStore: timeout after {t:.0f}s waiting for keys {list(keys)}")

    def delete_key(self, key):
        return self._client.delete(key)

    def num_keys(self):
        return self._client.num_keys()

    def append(self, key, value):
        self._client.append(key, _as_bytes(value))

    def set_timeout(self, timeout):
        self._timeout_s = timeout.total_seconds()

    # extras used by the framework -------------------------------------------------------------
    def try_get(self, key, timeout_s: float = 0.0):
        return self._client.try_get(key, timeout_s)

    def close(self):
        self._client.close()


def _as_bytes(v) -> bytes:
    if isinstance(v, bytes):
        return v
    if isinstance(v, str):
        return v.encode()
    return bytes(v)
