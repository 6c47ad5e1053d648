"""Fused flat AdamW (``csrc/adam.hip``).

Reference: the only optimizer step in the reference is DeepSpeed Adam inside
``model_engine.step()`` (``test/ccl.py:114-115``). Here the whole model's fp32 master
parameters, moments and (reduced) gradients are single flat buffers and one kernel updates them
and refreshes the bf16 working copy.
"""

from __future__ import annotations

from typing import Optional

import torch

from . import _lib
from ._lib import check, dt, use_hip


class FlatAdamW:
    def __init__(self, master: torch.Tensor, lr: float = 3e-4, betas=(0.9, 0.95),
                 eps: float = 1e-8, weight_decay: float = 0.0):
        if master.dtype != torch.float32 or not master.is_contiguous():
            raise ValueError("FlatAdamW master must be contiguous fp32")
        self.p = master
        self.m = torch.zeros_like(master)
        self.v = torch.zeros_like(master)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.t = 0

    @torch.no_grad()
    def step(self, grad: torch.Tensor, working_bf16: Optional[torch.Tensor] = None,
             grad_scale: float = 1.0) -> None:
        self.t += 1
        b1, b2 = self.betas
        if grad.numel() != self.p.numel():
            raise ValueError("grad / master size mismatch")
        if use_hip(self.p, grad):
            check(_lib.lib().dlbb_adamw(
                self.p.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), grad.data_ptr(),
                dt(grad), _lib.ptr(working_bf16), self.p.numel(), self.lr, b1, b2, self.eps,
                self.wd, self.t, float(grad_scale), _lib.stream(self.p.device)), "adamw")
            return
        g = grad.float() * grad_scale
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** self.t
        bc2 = 1 - b2 ** self.t
        denom = (self.v / bc2).sqrt_().add_(self.eps)
        self.p.mul_(1 - self.lr * self.wd).addcdiv_(self.m, denom, value=-self.lr / bc1)
        if working_bf16 is not None:
            working_bf16.copy_(self.p.to(working_bf16.dtype))
