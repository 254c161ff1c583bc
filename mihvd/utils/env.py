"""Process-topology discovery (rank / size / local rank) from the launcher environment.

The reference is launched by ``mpirun`` (horovod/tensorflow-mnist.yaml:17-38), which exports
``OMPI_COMM_WORLD_*``. mihvd accepts, in priority order:

1. mihvd/torchrun native variables: ``RANK``, ``WORLD_SIZE``, ``LOCAL_RANK``,
   ``LOCAL_WORLD_SIZE`` (+ ``MASTER_ADDR``/``MASTER_PORT``);
2. Open MPI: ``OMPI_COMM_WORLD_RANK/SIZE/LOCAL_RANK/LOCAL_SIZE``;
3. PMI / MPICH / Slurm-PMI: ``PMI_RANK``, ``PMI_SIZE`` (+ ``MPI_LOCALRANKID``/``MPI_LOCALNRANKS``);
4. nothing: a single process (rank 0 of 1).
"""
from __future__ import annotations

import dataclasses
import os
import socket


@dataclasses.dataclass(frozen=True)
class Topology:
    rank: int
    size: int
    local_rank: int
    local_size: int
    cross_rank: int
    cross_size: int
    master_addr: str
    master_port: int | None
    source: str


def _geti(env, *names, default=None):
    for n in names:
        v = env.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def discover(env=None) -> Topology:
    env = os.environ if env is None else env
    if env.get("RANK") is not None and env.get("WORLD_SIZE") is not None:
        source = "native"
        rank = _geti(env, "RANK")
        size = _geti(env, "WORLD_SIZE")
        local_rank = _geti(env, "LOCAL_RANK", default=rank)
        local_size = _geti(env, "LOCAL_WORLD_SIZE", "LOCAL_SIZE", default=size)
    elif env.get("OMPI_COMM_WORLD_RANK") is not None:
        source = "ompi"
        rank = _geti(env, "OMPI_COMM_WORLD_RANK")
        size = _geti(env, "OMPI_COMM_WORLD_SIZE", default=1)
        local_rank = _geti(env, "OMPI_COMM_WORLD_LOCAL_RANK", default=rank)
        local_size = _geti(env, "OMPI_COMM_WORLD_LOCAL_SIZE", default=size)
    elif env.get("PMI_RANK") is not None:
        source = "pmi"
        rank = _geti(env, "PMI_RANK")
        size = _geti(env, "PMI_SIZE", default=1)
        local_rank = _geti(env, "MPI_LOCALRANKID", "PMI_LOCAL_RANK", default=rank)
        local_size = _geti(env, "MPI_LOCALNRANKS", "PMI_LOCAL_SIZE", default=size)
    else:
        source = "single"
        rank, size, local_rank, local_size = 0, 1, 0, 1
    if not (0 <= rank < size):
        raise ValueError(f"invalid rank {rank} for world size {size} (from {source} env)")
    if not (0 <= local_rank < local_size):
        raise ValueError(f"invalid local rank {local_rank} for local size {local_size}")
    if size % local_size != 0:
        # heterogeneous hosts: cross-rank grouping still works by node index
        pass
    cross_rank = _geti(env, "GROUP_RANK", "MIHVD_CROSS_RANK", default=rank // max(1, local_size))
    cross_size = _geti(env, "MIHVD_CROSS_SIZE", default=max(1, (size + local_size - 1) // local_size))
    addr = env.get("MASTER_ADDR") or env.get("MIHVD_MASTER_ADDR") or "127.0.0.1"
    port = _geti(env, "MASTER_PORT", "MIHVD_MASTER_PORT", default=None)
    return Topology(rank, size, local_rank, local_size, cross_rank, cross_size, addr, port, source)


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]
