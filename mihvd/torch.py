"""Horovod-PyTorch-compatible API surface: ``import mihvd.torch as hvd``.

Everything the reference's entrypoints call through ``horovod.tensorflow`` /
``horovod.tensorflow.keras`` is available here for PyTorch-ROCm models.
"""
from .basics import (Adasum, Average, Max, Min, Product, ReduceOp, Sum, backend, ccl_built, config, cross_rank,
                     cross_size, cuda_built, ddl_built, device, engine_running, gloo_built, gloo_enabled, init, is_homogeneous,
                     is_initialized, local_rank, local_size, mpi_built, mpi_enabled, mpi_threads_supported, nccl_built,
                     rank, rccl_built, rocm_built, shutdown, size, start_timeline, stop_timeline, suspend_engine)
from .parallel.collectives import (allgather, allgather_async, allgather_object, allreduce, allreduce_,
                                   allreduce_async, allreduce_async_, alltoall, alltoall_async, barrier, broadcast,
                                   broadcast_, broadcast_async, broadcast_async_, broadcast_object, grouped_allgather,
                                   grouped_allgather_async, grouped_allreduce, grouped_allreduce_,
                                   grouped_allreduce_async, grouped_allreduce_async_,
                                   grouped_reducescatter, grouped_reducescatter_async, join, poll, reducescatter,
                                   reducescatter_async, sparse_allreduce_async, synchronize)
from .parallel.compression import Compression
from .parallel.optimizer import (DistributedOptimizer, PartialDistributedOptimizer, broadcast_optimizer_state,
                                 broadcast_parameters)
from .ops import collective_ops as mpi_ops  # noqa: E402,F401  registers torch.ops.mihvd_dist.* (Horovod's mpi_ops)
from . import elastic  # noqa: E402,F401  hvd.elastic.run / TorchState / ObjectState
from .process_sets import (ProcessSet, add_process_set, get_process_set_ids_and_ranks,  # noqa: E402,F401
                           global_process_set, remove_process_set)
from torch.nn import SyncBatchNorm  # noqa: E402,F401  (hvd.SyncBatchNorm: batch statistics over the process group)
