"""Data-parallel engine: collectives, fusion-bucketed DistributedOptimizer, Adasum, compression."""
from .collectives import (allgather, allgather_async, allgather_object, allreduce, allreduce_, allreduce_async,
                          allreduce_async_, alltoall, barrier, broadcast, broadcast_, broadcast_async,
                          broadcast_async_, broadcast_object, grouped_allreduce, join, poll, reducescatter,
                          synchronize)
from .compression import Compression
from .optimizer import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters

__all__ = [
    "allgather", "allgather_async", "allgather_object", "allreduce", "allreduce_", "allreduce_async",
    "allreduce_async_", "alltoall", "barrier", "broadcast", "broadcast_", "broadcast_async", "broadcast_async_",
    "broadcast_object", "grouped_allreduce", "join", "poll", "reducescatter", "synchronize", "Compression",
    "DistributedOptimizer", "broadcast_optimizer_state", "broadcast_parameters",
]
