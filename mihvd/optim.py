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
            lr_t = group["lr"] * math.sqrt(1 - b2 ** step_t) / (1 - b1 ** step_t)
            torch._foreach_mul_(ms, b1)
            torch._foreach_add_(ms, grads, alpha=1 - b1)
            torch._foreach_mul_(vs, b2)
            torch._foreach_addcmul_(vs, grads, grads, value=1 - b2)
            denom = torch._foreach_sqrt(vs)
            torch._foreach_add_(denom, group["eps"])
            torch._foreach_addcdiv_(params, ms, denom, value=-lr_t)
        return loss
