"""Direct xGMI one-shot allreduce (SURVEY.md §2.3 N4 "optional xGMI direct allreduce", §5.8).

RCCL's ring/tree allreduce pays one link latency per hop; for the small, latency-bound gradient
buckets of a B=100 MNIST step (horovod/tensorflow_mnist.py:133 reduces 8 tensors every step, all
but ``dense/kernel`` under 250 KB) a one-shot exchange over the fully connected xGMI mesh of an
MI355X node is shorter: every rank publishes its buffer, waits at a device-side barrier, then
reads all peers' buffers over its own point-to-point links and sums them in rank order
(``csrc/kernels/xgmi.hip``). No host involvement per call, so it can be captured in a HIP graph.

    ar = XGMIAllreduce(capacity_numel=1 << 20)       # collective: every rank of the group
    ar.allreduce_(t, average=True)                   # fp32, contiguous, numel <= capacity
    ar.check()                                       # raises if a device-side barrier timed out

Opt-in: the fused trainer uses it for its small-gradient bucket with ``MIHVD_XGMI_ALLREDUCE=1``;
``scripts/allreduce_bw.py --xgmi`` compares it against RCCL. Every rank of the group must sit on
one node (IPC handles), at most 8 ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops as _ops


class XGMIAllreduce:
    def __init__(self, capacity_numel: int, group=None, device: torch.device | None = None):
        if not dist.is_initialized():
            raise RuntimeError("XGMIAllreduce needs an initialised process group")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 8:
            raise ValueError("XGMIAllreduce supports at most 8 ranks (one MI355X node)")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.capacity = int(capacity_numel)
        o = _ops.load()
        self._o = o
        self.ctx = int(o.xgmi_create(self.device.index, self.capacity, self.rank, self.world))
        mine = o.xgmi_handle(self.ctx)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(mine.numpy().tobytes()), group=group)
        table = torch.frombuffer(bytearray(b"".join(handles)), dtype=torch.uint8).view(self.world, -1).clone()
        o.xgmi_open(self.ctx, table)
        dist.barrier(group=group)  # every peer has opened every buffer before the first signal
        self._closed = False

    def allreduce_(self, t: torch.Tensor, average: bool = False, scale: float = 1.0) -> torch.Tensor:
        """In-place sum (or average) of ``t`` over the group, on the current stream."""
        s = scale / self.world if average else scale
        self._o.xgmi_allreduce_(self.ctx, t, s)
        return t

    def check(self):
        """Synchronise the device and raise if any device-side barrier timed out."""
        err = int(self._o.xgmi_error(self.ctx))
        if err:
            raise RuntimeError(f"xGMI allreduce barrier timed out waiting for peers (mask {err:#x})")

    def close(self):
        if not self._closed:
            self._o.xgmi_destroy(self.ctx)
            self._closed = True
