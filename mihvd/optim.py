"""Optimizers with the reference's exact update rules.

``TFAdam`` implements ``tf.train.AdamOptimizer`` (horovod/tensorflow_mnist.py:130), which differs
from ``torch.optim.Adam`` in where epsilon sits:

    lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t)
    m    = beta1 * m + (1 - beta1) * g
    v    = beta2 * v + (1 - beta2) * g^2
    p   -= lr_t * m / (sqrt(v) + epsilon)          # epsilon = 1e-8 ("epsilon hat")

(Keras ``Adam`` — tensorflow_mnist_gpu.py:134 — is the same rule with epsilon 1e-7.) The state
names match torch's Adam (``exp_avg``, ``exp_avg_sq``, ``step``) so checkpoint mapping and
``broadcast_optimizer_state`` work unchanged. The fused HIP kernel ``mihvd::adam_step`` uses the
identical rule on the flat parameter buffer.
"""
from __future__ import annotations

import math

import torch


def _fused_ok(tensors) -> bool:
    """The multi-tensor HIP kernels apply: every tensor is a contiguous fp32 GPU tensor."""
    if not tensors or not all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in tensors):
        return False
    from . import _native

    return _native.load_kernels()


def _dense(t: torch.Tensor) -> bool:
    if t.is_contiguous():
        return True
    if t.dim() == 4:
        return t.is_contiguous(memory_format=torch.channels_last)
    if t.dim() == 5:
        return t.is_contiguous(memory_format=torch.channels_last_3d)
    return False


def _flat(t: torch.Tensor) -> torch.Tensor:
    return t.as_strided((t.numel(),), (1,), t.storage_offset())


def _split_fused(*lists):
    """Partition parallel tensor lists (p, g, state...) into the ones the multi-tensor kernels can
    update — fp32 GPU tensors that are dense with identical strides (e.g. channels_last conv
    weights whose grads and slots share the layout), passed as flat views — and the indices left
    to the torch path."""
    from . import _native

    n = len(lists[0])
    ok_kernels = n > 0 and lists[0][0].is_cuda and _native.load_kernels()
    fused = [[] for _ in lists]
    rest = []
    for i in range(n):
        ts = [lst[i] for lst in lists]
        good = ok_kernels and all(
            t.is_cuda and t.dtype == torch.float32 and t.stride() == ts[0].stride() and t.shape == ts[0].shape
            and _dense(t) for t in ts)
        if good:
            for f, t in zip(fused, ts):
                f.append(_flat(t))
        else:
            rest.append(i)
    return fused, rest


class TFAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        if lr < 0:
            raise ValueError("invalid learning rate")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            params, grads, ms, vs = [], [], [], []
            step_t = None
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                step_t = float(st["step"])
                params.append(p)
                grads.append(p.grad)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
            if not params:
                continue
            if _fused_ok(params + grads + ms + vs):
                # one multi-tensor HIP launch per 24 tensors (csrc/kernels/multi_tensor.hip), same rule
                torch.ops.mihvd.multi_tensor_adam(params, grads, ms, vs, None, int(step_t), group["lr"], b1, b2,
                                                  group["eps"], 0.0, False, 0, 1.0)
                continue
            lr_t = group["lr"] * math.sqrt(1 - b2 ** step_t) / (1 - b1 ** step_t)
            torch._foreach_mul_(ms, b1)
            torch._foreach_add_(ms, grads, alpha=1 - b1)
            torch._foreach_mul_(vs, b2)
            torch._foreach_addcmul_(vs, grads, grads, value=1 - b2)
            denom = torch._foreach_sqrt(vs)
            torch._foreach_add_(denom, group["eps"])
            torch._foreach_addcdiv_(params, ms, denom, value=-lr_t)
        return loss


class FusedAdam(torch.optim.Optimizer):
    """Adam / AdamW over arbitrary parameter lists with the multi-tensor HIP kernel.

    ``rule="torch"`` is torch.optim.Adam's update, ``rule="tf"`` the TF1 rule of ``TFAdam``;
    ``adamw=True`` decouples the weight decay. The step count of each parameter group lives in a
    device int64 tensor advanced by a tiny kernel, so ``step()`` issues no host synchronisation and
    can be captured in a HIP graph (``mihvd.graphs.CapturedStep``). Checkpoints carry the count as
    ``param_groups[i]["step"]``. Falls back to torch ops for CPU tensors.
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=False, rule="torch"):
        if rule not in ("torch", "tf"):
            raise ValueError("rule must be 'torch' or 'tf'")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=adamw, rule=rule,
                                      step=0))
        self._dev_steps: dict[int, torch.Tensor] = {}

    def _group_step(self, gi, group, device):
        t = self._dev_steps.get(gi)
        if t is None or t.device != device:
            t = torch.full((1,), int(group.get("step", 0)), dtype=torch.int64, device=device)
            self._dev_steps[gi] = t
        return t

    def state_dict(self):
        for gi, group in enumerate(self.param_groups):
            if gi in self._dev_steps:
                group["step"] = int(self._dev_steps[gi].item())
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for gi, group in enumerate(self.param_groups):
            if gi in self._dev_steps:
                self._dev_steps[gi].fill_(int(group.get("step", 0)))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                st = self.state[p]
                if not st:
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            grads = [p.grad for p in params]
            ms = [self.state[p]["exp_avg"] for p in params]
            vs = [self.state[p]["exp_avg_sq"] for p in params]
            b1, b2 = group["betas"]
            rule = 0 if group["rule"] == "tf" else 1
            from . import _native

            if params[0].is_cuda and _native.load_kernels():
                stp = self._group_step(gi, group, params[0].device)
                torch.ops.mihvd.bump_step_(stp)
                (fp, fg, fm, fv), idx = _split_fused(params, grads, ms, vs)
                if fp:
                    torch.ops.mihvd.multi_tensor_adam(fp, fg, fm, fv, stp, 0, group["lr"], b1, b2, group["eps"],
                                                      group["weight_decay"], bool(group["adamw"]), rule, 1.0)
                if not idx:
                    continue
                t = int(stp.item())  # tensors the kernel cannot take: torch path (one host read)
            else:
                group["step"] = int(group.get("step", 0)) + 1
                t = group["step"]
                idx = range(len(params))
            bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
            for i in idx:
                p, g, m, v = params[i], grads[i], ms[i], vs[i]
                if group["weight_decay"]:
                    if group["adamw"]:
                        p.mul_(1 - group["lr"] * group["weight_decay"])
                    else:
                        g = g.add(p, alpha=group["weight_decay"])
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                if rule == 0:
                    p.addcdiv_(m, v.sqrt().add_(group["eps"]), value=-group["lr"] * math.sqrt(bc2) / bc1)
                else:
                    p.addcdiv_(m, (v / bc2).sqrt().add_(group["eps"]), value=-group["lr"] / bc1)
        return loss


class FusedSGD(torch.optim.Optimizer):
    """SGD with momentum / dampening / Nesterov / weight decay (torch.optim.SGD semantics) with the
    multi-tensor HIP kernel; no host synchronisation after the first step (capturable)."""

    def __init__(self, params, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            mom = group["momentum"]
            first = False
            bufs = []
            if mom:
                for p in params:
                    st = self.state[p]
                    if "momentum_buffer" not in st:
                        st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                        first = True  # the group's buffers are created together, on its first step
                    bufs.append(st["momentum_buffer"])
            grads = [p.grad for p in params]
            if mom:
                (fp, fg, fb), idx = _split_fused(params, grads, bufs)
            else:
                (fp, fg), idx = _split_fused(params, grads)
                fb = []
            if fp:
                torch.ops.mihvd.multi_tensor_sgd(fp, fg, fb, group["lr"], mom, group["dampening"],
                                                 group["weight_decay"], bool(group["nesterov"]), first, 1.0)
            for i in idx:
                p, g = params[i], grads[i]
                d = g.add(p, alpha=group["weight_decay"]) if group["weight_decay"] else g
                if mom:
                    b = bufs[i]
                    if first:
                        b.copy_(d)
                    else:
                        b.mul_(mom).add_(d, alpha=1 - group["dampening"])
                    d = d.add(b, alpha=mom) if group["nesterov"] else b
                p.add_(d, alpha=-group["lr"])
        return loss
