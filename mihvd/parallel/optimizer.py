"""``DistributedOptimizer`` and state broadcast (Horovod torch API).

Reference call sites: ``hvd.DistributedOptimizer(opt, op=hvd.Adasum if args.use_adasum else
hvd.Average)`` (horovod/tensorflow_mnist.py:133, tensorflow_mnist_gpu.py:137-138) and
``hvd.BroadcastGlobalVariablesHook(0)`` (tensorflow_mnist.py:143).

Design (SURVEY.md §2.3 N1-N3, §5.8 "Overlap"):

* At construction the native ``plan_buckets`` lays every gradient out in a few flat, 256-byte
  aligned fusion buffers, in reverse registration order (≈ the order backward produces them), and
  each ``param.grad`` becomes a *view* into its bucket — zero-copy fusion, no pack/unpack pass.
* A post-accumulate-grad hook per parameter feeds the native ``Controller``; whenever a bucket is
  complete *and* every earlier bucket has been launched, its allreduce is issued asynchronously on
  the framework-owned RCCL communicator's high-priority stream (``collectives.BucketPlane``; the
  process group only on gloo or with ``MIHVD_COMM=torch``), overlapping the rest of backward.
  Strict in-order release is what gives all ranks the same collective order without Horovod's
  per-cycle negotiation.
* ``step()`` flushes buckets whose gradients never arrived (unused parameters), waits for all of
  them, then runs the wrapped optimizer.
"""
from __future__ import annotations

import contextlib
import warnings
from typing import Iterable

import torch
import torch.distributed as dist

from .. import basics
from ..basics import ReduceOp
from . import collectives as C
from ..utils.tracing import trace_range
from .compression import Compression

_DTYPE_CODES: dict[torch.dtype, int] = {}


def _dtype_code(dt: torch.dtype) -> int:
    if dt not in _DTYPE_CODES:
        _DTYPE_CODES[dt] = len(_DTYPE_CODES) + 1
    return _DTYPE_CODES[dt]


class _Bucket:
    __slots__ = ("index", "flat", "members", "offsets", "segments", "handle", "wire")

    def __init__(self, index, flat, members, offsets, segments, wire=None):
        self.index = index
        self.flat = flat
        self.members = members
        self.offsets = offsets
        self.segments = segments
        self.handle = None
        # persistent 16-bit wire buffer of a compressed bucket: no allocation per step (and none
        # inside a captured HIP graph, whose private pool would otherwise own it)
        self.wire = wire


class _DistributedOptimizer(torch.optim.Optimizer):
    """Mixin body; instances are created through :func:`DistributedOptimizer`."""

    def _mihvd_setup(self, named_parameters, compression, backward_passes_per_step, op,
                     gradient_predivide_factor, fusion_threshold, sparse_as_dense, local_params=()):
        from .._native import runtime

        basics._require()
        local = {id(p) for p in local_params}  # PartialDistributedOptimizer: never reduced
        self._compression = compression
        self._op = ReduceOp(op)
        self._predivide = float(gradient_predivide_factor)
        if self._predivide != 1.0 and self._op != ReduceOp.Average:
            raise ValueError("gradient_predivide_factor requires op=Average")
        self._passes = int(backward_passes_per_step)
        params = [p for g in self.param_groups for p in g["params"] if p.requires_grad and id(p) not in local]
        seen = set()
        uniq = []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        params = uniq
        names = {}
        if named_parameters is not None:
            named_parameters = list(named_parameters)
            if any(not isinstance(t, tuple) or len(t) != 2 for t in named_parameters):
                raise ValueError("named_parameters should be a sequence of (name, parameter) tuples")
            dups = {n for n, _ in named_parameters if sum(1 for m, _ in named_parameters if m == n) > 1}
            if dups:
                raise ValueError(f"parameter names must be unique; duplicates: {sorted(dups)}")
            names = {id(p): n for n, p in named_parameters if id(p) not in local}
            missing = [p for p in params if id(p) not in names]
            if missing:
                raise ValueError("named_parameters was specified, but one or more model parameters "
                                 "were not named")
        self._params = params
        # the framework-owned RCCL bucket plane (collective: every rank constructs its optimizer);
        # None on gloo / at size 1 / with MIHVD_COMM=torch: the engine or the process group then
        self._plane = C.bucket_plane() if any(p.is_cuda for p in params) else None
        self._names = [names.get(id(p), f"param.{i}") for i, p in enumerate(params)]
        self._index = {id(p): i for i, p in enumerate(params)}
        cfg = basics.config()
        thresh = cfg.fusion_threshold if fusion_threshold is None else int(fusion_threshold)
        self._tuner = None
        if cfg.autotune and fusion_threshold is None and basics.size() > 1:
            from .autotune import FusionAutotuner

            self._tuner = FusionAutotuner.from_config(cfg)
            thresh = self._tuner.first()
        self._plan(thresh)
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(params)]
        self._synchronized = False
        self._should_sync = True
        self._consistency_checked = not cfg.consistency_check
        if basics._ctx.elastic_gen is None:
            self._check_consistency()
        # elastic worlds: a worker joining mid-training constructs its optimizer while the others
        # are already training, so the (collective) check runs at the first synchronize() after
        # every re-formed world instead, where all ranks meet

    def _plan(self, thresh: int):
        """(Re)build the fusion buckets for ``thresh`` bytes and point every ``param.grad`` at its
        slot (current gradient values are carried over)."""
        from .._native import runtime

        params = self._params
        rt = runtime()
        specs = [rt.TensorSpec(p.numel(), p.element_size(), _dtype_code(p.dtype),
                               (p.device.index if p.device.index is not None else -1) if p.is_cuda else -2)
                 for p in params]
        order = list(range(len(params)))[::-1]
        plan = rt.plan_buckets(specs, order, int(thresh), basics.config().bucket_align) if params else None
        self._fusion_threshold = int(thresh)
        self._buckets: list[_Bucket] = []
        if plan is not None:
            for b in range(len(plan)):
                p0 = params[plan.members[b][0]]
                flat = torch.zeros(plan.numel[b], dtype=p0.dtype, device=p0.device)
                segs = [(int(o), int(o) + params[i].numel()) for i, o in zip(plan.members[b], plan.offsets[b])]
                wdt = getattr(self._compression, "wire_dtype", None)
                wire = (torch.empty(flat.numel(), dtype=wdt, device=flat.device)
                        if wdt is not None and flat.is_cuda and flat.dtype == torch.float32 else None)
                self._buckets.append(_Bucket(b, flat, list(plan.members[b]), list(plan.offsets[b]), segs, wire))
            self._tensor_bucket = list(plan.tensor_bucket)
            self._tensor_offset = list(plan.tensor_offset)
            self._controller = rt.Controller(self._tensor_bucket, len(self._buckets), self._passes)
            self._install_grad_views()
        else:
            self._controller = None

    # -- gradient views --------------------------------------------------------------------
    def _install_grad_views(self):
        for i, p in enumerate(self._params):
            b = self._buckets[self._tensor_bucket[i]]
            off = self._tensor_offset[i]
            view = b.flat[off:off + p.numel()].view_as(p)
            if p.grad is not None:
                view.copy_(p.grad)
            p.grad = view

    def _views_intact(self) -> bool:
        for i, p in enumerate(self._params):
            g = p.grad
            if g is None:
                return False
            b = self._buckets[self._tensor_bucket[i]]
            if g.data_ptr() != b.flat.data_ptr() + self._tensor_offset[i] * b.flat.element_size():
                return False
        return True

    def _check_consistency(self):
        if self._consistency_checked or basics.size() == 1:
            self._consistency_checked = True
            return
        from .._native import runtime

        sig = runtime().tensor_signature(self._names, [list(p.shape) for p in self._params],
                                         [str(p.dtype) for p in self._params])
        sigs = C.allgather_object(int(sig))
        if len(set(sigs)) != 1:
            raise RuntimeError(
                "mihvd: gradient tensors differ across ranks (name/shape/dtype signature mismatch: "
                f"{sigs}); every rank must build the same model and optimizer")
        self._consistency_checked = True

    # -- hooks and launches ----------------------------------------------------------------
    def _make_hook(self, idx):
        def hook(p):
            if not self._should_sync or self._controller is None:
                return
            g = p.grad
            if g is not None:
                b = self._buckets[self._tensor_bucket[idx]]
                expected = b.flat.data_ptr() + self._tensor_offset[idx] * b.flat.element_size()
                if g.data_ptr() != expected:
                    # The grad was replaced (e.g. zero_grad(set_to_none) outside our control):
                    # fold it back into the bucket view.
                    view = b.flat[self._tensor_offset[idx]:self._tensor_offset[idx] + p.numel()].view_as(p)
                    view.copy_(g)
                    p.grad = view
            for bid in self._controller.mark_ready(idx):
                self._launch(bid)
        return hook

    def _launch(self, bid: int):
        with trace_range(f"mihvd.bucket{bid}.allreduce"):
            self._launch_impl(bid)

    def _launch_impl(self, bid: int):
        b = self._buckets[bid]
        if self._op == ReduceOp.Average and self._predivide != 1.0:
            pre, post = 1.0 / self._predivide, self._predivide
        else:
            pre, post = 1.0, 1.0
        if self._op == ReduceOp.Adasum:
            b.handle = C._allreduce_impl(b.flat, b.flat, f"bucket{bid}", ReduceOp.Adasum, self._compression, pre,
                                         post, None, segments=b.segments)
        else:
            b.handle = C._allreduce_impl(b.flat, b.flat, f"bucket{bid}", self._op, self._compression, pre, post, None,
                                         wire_buf=b.wire, plane=self._plane if b.flat.is_cuda else None)

    def synchronize(self):
        """Launch any bucket not yet launched, then wait for every bucket's allreduce."""
        if self._controller is None:
            self._synchronized = True
            return
        if not self._views_intact():
            self._install_grad_views()
        if not self._consistency_checked:
            self._check_consistency()
        with trace_range("mihvd.synchronize"):
            for bid in self._controller.flush():
                self._launch(bid)
            for b in self._buckets:
                if b.handle is not None:
                    C.synchronize(b.handle)
                    b.handle = None
        self._controller.reset()
        self._synchronized = True

    @contextlib.contextmanager
    def skip_synchronize(self):
        """Use after an explicit ``synchronize()`` so ``step()`` does not wait again."""
        self._should_sync = False
        try:
            yield
        finally:
            self._should_sync = True

    def step(self, closure=None):
        if self._should_sync:
            if self._synchronized:
                warnings.warn("optimizer.step() called without a backward pass since the last synchronize()")
            self.synchronize()
        self._synchronized = False
        with trace_range("mihvd.optimizer_step"):
            out = super(self.__class__, self).step(closure)
        if self._tuner is not None:
            new = self._tuner.on_step()
            if new is not None and new != self._fusion_threshold:
                self._plan(new)
        return out

    def _elastic_reset(self):
        """Forget in-flight bucket allreduces of a step interrupted by a failed or re-formed world
        (mihvd.elastic): the next backward starts with every bucket un-launched, on the bucket plane
        of the NEW world (shutdown closed the old one; collective: every rank's State.sync() calls
        this)."""
        self._plane = C.bucket_plane() if any(p.is_cuda for p in self._params) else None
        if self._controller is not None:
            for b in self._buckets:
                b.handle = None
            self._controller.reset()
        self._synchronized = False
        self._consistency_checked = not basics.config().consistency_check

    @property
    def fusion_threshold(self) -> int:
        return self._fusion_threshold

    def zero_grad(self, set_to_none: bool = True):
        # Gradients live inside the fusion buffers: zero them in place and keep the views.
        if self._controller is not None:
            for b in self._buckets:
                if b.handle is not None:
                    raise AssertionError("zero_grad() called while allreduces are in flight; call step() "
                                         "or synchronize() first")
            for b in self._buckets:
                b.flat.zero_()
            if not self._views_intact():
                self._install_grad_views()
            reduced = {id(p) for p in self._params}
            for g in self.param_groups:  # parameters kept local (PartialDistributedOptimizer)
                for p in g["params"]:
                    if id(p) not in reduced and p.grad is not None:
                        if set_to_none:
                            p.grad = None
                        else:
                            p.grad.zero_()
        else:
            super(self.__class__, self).zero_grad(set_to_none)

    @property
    def buckets(self):
        return [(b.index, [self._names[i] for i in b.members], b.flat.numel(), b.flat.dtype) for b in self._buckets]


def DistributedOptimizer(optimizer: torch.optim.Optimizer, named_parameters=None, compression=Compression.none,
                         backward_passes_per_step: int = 1, op=ReduceOp.Average, gradient_predivide_factor=1.0,
                         fusion_threshold=None, sparse_as_dense=False, num_groups=0, groups=None, process_set=None):
    """Wrap ``optimizer`` so gradients are averaged (or Adasum-combined) across ranks before
    ``step()``. Returns an instance of a dynamic subclass of the optimizer's class, so it is still
    ``isinstance`` of the original optimizer type."""
    cls = type(optimizer.__class__.__name__, (optimizer.__class__,), dict(_DistributedOptimizer.__dict__))
    obj = cls.__new__(cls)
    obj.__dict__.update(optimizer.__dict__)
    obj._mihvd_setup(named_parameters, compression, backward_passes_per_step, op, gradient_predivide_factor,
                     fusion_threshold, sparse_as_dense)
    return obj


def PartialDistributedOptimizer(optimizer: torch.optim.Optimizer, named_parameters=None, compression=Compression.none,
                                backward_passes_per_step: int = 1, op=ReduceOp.Average, gradient_predivide_factor=1.0,
                                fusion_threshold=None, sparse_as_dense=False, local_layers=None, process_set=None):
    """Horovod's ``PartialDistributedOptimizer``: like :func:`DistributedOptimizer`, but the
    parameters of ``local_layers`` (modules, or an iterable of modules) keep their per-rank
    gradients — they are updated by the wrapped optimizer without any allreduce (e.g. rank-local
    heads or embeddings trained on rank-specific data)."""
    mods = [] if local_layers is None else (
        [local_layers] if isinstance(local_layers, torch.nn.Module) else list(local_layers))
    local_params = [p for m in mods for p in m.parameters()]
    cls = type(optimizer.__class__.__name__, (optimizer.__class__,), dict(_DistributedOptimizer.__dict__))
    obj = cls.__new__(cls)
    obj.__dict__.update(optimizer.__dict__)
    obj._mihvd_setup(named_parameters, compression, backward_passes_per_step, op, gradient_predivide_factor,
                     fusion_threshold, sparse_as_dense, local_params=local_params)
    return obj


# ------------------------------------------------------------------------------------------ #
# State broadcast
# ------------------------------------------------------------------------------------------ #
def _flat_broadcast_(tensors: list[torch.Tensor], root_rank: int):
    """Broadcast tensors in place with one collective per (dtype, device) group."""
    if basics.size() == 1 or not tensors:
        return
    groups: dict[tuple, list[torch.Tensor]] = {}
    for t in tensors:
        groups.setdefault((t.dtype, t.device), []).append(t)
    dev = basics.device()
    for (dt, d), ts in groups.items():
        flat = torch.cat([t.detach().reshape(-1).to(dev) for t in ts])
        C.broadcast_(flat, root_rank, name="params")
        off = 0
        for t in ts:
            n = t.numel()
            with torch.no_grad():
                t.copy_(flat[off:off + n].view_as(t))
            off += n


def broadcast_parameters(params, root_rank: int = 0):
    """Broadcast a ``state_dict()``, ``named_parameters()`` list or module from ``root_rank``."""
    basics._require()
    if isinstance(params, torch.nn.Module):
        params = params.state_dict()
    if isinstance(params, dict):
        items = sorted(params.items(), key=lambda kv: kv[0])
    else:
        items = list(params)
    tensors = []
    for name, t in items:
        if t is None or not torch.is_tensor(t):
            continue
        tensors.append(t.data if isinstance(t, torch.nn.Parameter) else t)
    _flat_broadcast_(tensors, root_rank)


def _split_state(obj, tensors):
    if torch.is_tensor(obj):
        tensors.append(obj)
        return {"__mihvd_tensor__": len(tensors) - 1, "shape": list(obj.shape), "dtype": str(obj.dtype).replace("torch.", ""),
                "device_is_cpu": obj.device.type == "cpu"}
    if isinstance(obj, dict):
        return {k: _split_state(v, tensors) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_split_state(v, tensors) for v in obj)
    return obj


def _join_state(meta, tensors):
    if isinstance(meta, dict) and "__mihvd_tensor__" in meta:
        return tensors[meta["__mihvd_tensor__"]]
    if isinstance(meta, dict):
        return {k: _join_state(v, tensors) for k, v in meta.items()}
    if isinstance(meta, (list, tuple)):
        return type(meta)(_join_state(v, tensors) for v in meta)
    return meta


def broadcast_optimizer_state(optimizer: torch.optim.Optimizer, root_rank: int = 0):
    """Broadcast optimizer state (e.g. Adam ``exp_avg``/``exp_avg_sq``/``step``) and
    hyper-parameters from ``root_rank`` — the optimizer half of ``BroadcastGlobalVariablesHook``."""
    basics._require()
    if basics.size() == 1:
        return
    sd = optimizer.state_dict()
    local_tensors: list[torch.Tensor] = []
    meta = _split_state(sd, local_tensors)
    meta = C.broadcast_object(meta, root_rank)
    # Allocate receive buffers from the root's metadata (ranks with empty state get zeros).
    specs = []

    def collect(m):
        if isinstance(m, dict) and "__mihvd_tensor__" in m:
            specs.append(m)
        elif isinstance(m, dict):
            for v in m.values():
                collect(v)
        elif isinstance(m, (list, tuple)):
            for v in m:
                collect(v)

    collect(meta)
    specs.sort(key=lambda m: m["__mihvd_tensor__"])
    dev = basics.device()
    bufs = []
    for m in specs:
        i = m["__mihvd_tensor__"]
        dt = getattr(torch, m["dtype"])
        if basics.rank() == root_rank:
            t = local_tensors[i]
        else:
            t = torch.zeros(m["shape"], dtype=dt)
        bufs.append(t)
    work = [t.to(dev) for t in bufs]
    _flat_broadcast_(work, root_rank)
    out = [w.cpu() if m["device_is_cpu"] else w for w, m in zip(work, specs)]
    optimizer.load_state_dict(_join_state(meta, out))
