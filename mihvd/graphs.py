"""Whole-step HIP-graph capture for models trained through the generic engine.

The fused MNIST trainer replays its hand-written kernels from a HIP graph. ``CapturedStep`` does
the same for any PyTorch model: forward, backward (whose gradient hooks launch the
DistributedOptimizer's bucket allreduces — RCCL calls are captured), the allreduce waits and a
capturable optimizer (``mihvd.optim.FusedAdam`` / ``FusedSGD``: device-side step count, no host
synchronisation) become one graph that the host launches with a single call — the MI355X
replacement for a tracing compiler on launch-bound models.

    x, y = static input buffers (copy each batch into them, or gather on the device)
    def step():
        opt.zero_grad(set_to_none=False)
        loss = loss_fn(model(x), y)
        loss.backward()
        opt.step()
        return loss
    graphed = CapturedStep(step)        # warm-up runs + capture
    for batch in data:
        x.copy_(batch.x); y.copy_(batch.y)
        loss = graphed()                # replay

Tensors the step allocates are owned by the graph's private memory pool and are overwritten by the
next replay; ``graphed()`` returns the step's (static) output.
"""
from __future__ import annotations

import os

import torch


class CapturedStep:
    """``serialize=True``: each replay is launched only once the previous one has completed (a
    host wait on an event; costs one launch latency per step)."""

    def __init__(self, step_fn, warmup: int = 3, pool=None, serialize: bool = False, sync_warmup: bool = True):
        if not torch.cuda.is_available():
            raise RuntimeError("CapturedStep needs a GPU")
        self.step_fn = step_fn
        self.serialize = bool(serialize)
        self._done = torch.cuda.Event() if self.serialize else None
        self._pending = False
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        # The last warm-up step's output, autograd graph included, stays alive for the life of the
        # captured step, and each warm-up output is read back before the next step is issued. With
        # the warm-up freed before capture instead, BERT-base's replays go non-finite at the second
        # replay once the host synchronises between replays (scripts/bert_graph_bisect.py: variants
        # H vs C, and this class with MIHVD_GRAPH_HOLD_WARMUP=0); held, they track eager. Costs one
        # step's activations of memory. MIHVD_GRAPH_HOLD_WARMUP=0 restores the freeing form.
        hold = os.environ.get("MIHVD_GRAPH_HOLD_WARMUP", "1") != "0"
        self._held = None
        with torch.cuda.stream(side):  # warm-up on a side stream, as graph capture of autograd requires
            for _ in range(warmup):
                out = step_fn()
                if hold:
                    _readback(out)
                    self._held = out
                else:
                    _detach(out)  # drop the autograd graph: no AccumulateGrad node outlives its step
                del out
                if sync_warmup:
                    # each warm-up step completes before the next is issued (scripts/bert_graph_bisect.py:
                    # variant H vs C)
                    side.synchronize()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool):
            self.output = _detach(step_fn())
        self.replays = 0

    def __call__(self):
        if self._pending:
            self._done.synchronize()
        self.graph.replay()
        if self.serialize:
            self._done.record()
            self._pending = True
        self.replays += 1
        return self.output

    def pool(self):
        return self.graph.pool()


def _readback(out):
    """Copy one element of the first tensor in ``out`` to the host (synchronising its stream)."""
    if torch.is_tensor(out):
        if out.numel():
            out.detach().reshape(-1)[:1].cpu()
        return True
    if isinstance(out, (list, tuple)):
        return any(_readback(o) for o in out)
    if isinstance(out, dict):
        return any(_readback(o) for o in out.values())
    return False


def _detach(out):
    if torch.is_tensor(out):
        return out.detach()
    if isinstance(out, (list, tuple)):
        return type(out)(_detach(o) for o in out)
    if isinstance(out, dict):
        return {k: _detach(v) for k, v in out.items()}
    return out
