"""mihvd — an MI355X-native data-parallel training framework with a Horovod-style API.

``import mihvd.torch as hvd`` gives the Horovod PyTorch surface (``init``, ``rank``, ``size``,
``local_rank``, ``local_size``, ``DistributedOptimizer``, ``broadcast_parameters``, ...);
``mihvd.tensorflow`` and ``mihvd.keras`` give the TF1-hook and Keras-callback shaped APIs used by
the reference's two entrypoints (horovod/tensorflow_mnist.py, horovod/tensorflow_mnist_gpu.py).

Packages: ``parallel`` (RCCL collectives, fusion buckets, Adasum), ``ops`` (hand-written CDNA4 HIP
kernels), ``models`` (MNIST CNN: reference-semantics torch model + fused HIP training step),
``utils`` (env discovery, checkpoints, data, logging, timeline), ``runner`` (``mihvdrun``).
"""
from .basics import (Adasum, Average, Max, Min, Product, ReduceOp, Sum, backend, ccl_built, config, cross_rank,
                     cross_size, cuda_built, ddl_built, device, engine_running, gloo_built, gloo_enabled, init, is_homogeneous,
                     is_initialized, local_rank, local_size, mpi_built, mpi_enabled, mpi_threads_supported, nccl_built,
                     rank, rccl_built, rocm_built, shutdown, size, start_timeline, stop_timeline, suspend_engine)

__version__ = "0.1.0"
