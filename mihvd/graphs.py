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
    host wait on an event; costs one launch latency per step).

    The parameters' ``AccumulateGrad`` nodes — the autograd nodes that add each backward's gradient
    into ``p.grad`` — are kept alive from the warm-up through the capture (``self.accumulators``),
    so the captured backward accumulates through the same nodes the warm-up created instead of
    nodes created while capturing. Autograd holds a leaf's node only weakly: once the last warm-up
    step's graph is freed the node dies and the capture's forward builds a new one. With the new
    nodes, BERT-base under bf16 autocast replays correctly once and then writes non-finite values
    into the Linear layers' bias gradients from the second replay on (scripts/bert_graph_bisect.py:
    variant C0 fails, A0 — C0 holding only these nodes — tracks eager; fp32 (N) is unaffected;
    profiles/r04/bert_graph_bisect_*.log). Holding the nodes costs no activation memory: a leaf's
    node references the parameter, not the step's tensors. ``MIHVD_GRAPH_HOLD_ACCUMULATORS=0``
    restores the failing form for study.

    What the bisection pins down: the failing captures accumulate each bias gradient (a bf16 sum
    over the batch, cast to fp32) on the stream that produced it; every passing form hands it to an
    AccumulateGrad on another stream behind an event (A0) or has no cast node on the bias path (F0,
    bias added in fp32). Nothing runs eagerly during the capture and no ``.grad`` tensor is swapped
    for another (both checked per parameter), so the stale read is inside the graph's own replay of
    autograd's same-stream accumulation path.
    """

    def __init__(self, step_fn, warmup: int = 3, pool=None, serialize: bool = False, sync_warmup: bool = False,
                 params=None):
        if not torch.cuda.is_available():
            raise RuntimeError("CapturedStep needs a GPU")
        self.step_fn = step_fn
        self.serialize = bool(serialize)
        self._done = torch.cuda.Event() if self.serialize else None
        self._pending = False
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        hold = os.environ.get("MIHVD_GRAPH_HOLD_ACCUMULATORS", "1") != "0"
        self.accumulators = []
        with torch.cuda.stream(side):  # warm-up on a side stream, as graph capture of autograd requires
            for i in range(warmup):
                out = step_fn()
                if hold and i == warmup - 1:
                    # the nodes of the warm-up graph (step_fn returns a tensor with a grad_fn), or
                    # those of ``params`` directly (a step that returns loss.detach(), a float, None)
                    self.accumulators = (param_accumulate_grad_nodes(params) if params is not None
                                         else accumulate_grad_nodes(out))
                    if not self.accumulators:
                        import warnings

                        warnings.warn("CapturedStep: no AccumulateGrad node found to hold (step_fn returned "
                                      "no tensor with a grad_fn; pass params=): the capture re-creates them, "
                                      "the form that replays stale gradient reads (see the class docstring)")
                _detach(out)
                del out
                if sync_warmup:
                    side.synchronize()  # each warm-up step completes before the next is issued
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # Captured on torch's capture stream, not on `side`: the held nodes then accumulate on their
        # own stream behind an event, which replays correctly; capturing on `side` itself (variant AR
        # of scripts/bert_graph_bisect.py) fails like freshly created nodes do. That stream mismatch
        # is the point, so autograd's warning about it is switched off for the capture.
        warn = _stream_mismatch_warning(False) if self.accumulators else None
        try:
            with torch.cuda.graph(self.graph, pool=pool):
                self.output = _detach(step_fn())
        finally:
            if warn is not None:
                _stream_mismatch_warning(warn)
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


def _stream_mismatch_warning(on: bool):
    """Set autograd's AccumulateGrad stream-mismatch warning; returns the previous setting."""
    g = torch.autograd.graph
    if not hasattr(g, "set_warn_on_accumulate_grad_stream_mismatch"):
        return None
    prev = bool(torch._C._warn_on_accumulate_grad_stream_mismatch()) if hasattr(
        torch._C, "_warn_on_accumulate_grad_stream_mismatch") else True
    g.set_warn_on_accumulate_grad_stream_mismatch(bool(on))
    return prev


def param_accumulate_grad_nodes(params):
    """The ``AccumulateGrad`` node of every leaf tensor in ``params`` that requires grad (the node
    autograd keeps for the leaf, reached through a view's backward)."""
    found = []
    for p in params:
        if torch.is_tensor(p) and p.requires_grad and p.grad_fn is None:
            node = p.view_as(p).grad_fn.next_functions[0][0]
            if node is not None:
                found.append(node)
    return found


def accumulate_grad_nodes(out):
    """Every ``AccumulateGrad`` node reachable from the autograd graph of the tensors in ``out``
    (a tensor, or a list / tuple / dict of them). The graph's saved tensors may already be freed
    (after ``backward()``): only the node objects are walked."""
    stack, seen, found, alive = [], set(), [], []

    def roots(o):
        if torch.is_tensor(o):
            if o.grad_fn is not None:
                stack.append(o.grad_fn)
        elif isinstance(o, (list, tuple)):
            for x in o:
                roots(x)
        elif isinstance(o, dict):
            for x in o.values():
                roots(x)

    roots(out)
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        seen.add(id(fn))
        alive.append(fn)  # keeps the wrapper alive: a freed wrapper's id() can be reused by the next one
        if hasattr(fn, "variable"):  # torch::autograd::AccumulateGrad
            found.append(fn)
        for nxt, _ in fn.next_functions:
            stack.append(nxt)
    return found


def _detach(out):
    if torch.is_tensor(out):
        return out.detach()
    if isinstance(out, (list, tuple)):
        return type(out)(_detach(o) for o in out)
    if isinstance(out, dict):
        return {k: _detach(v) for k, v in out.items()}
    return out
