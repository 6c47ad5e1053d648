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
        self.t_dev: Optional[torch.Tensor] = None   # device step counter (HIP-graph mode)

    def enable_device_step(self) -> None:
        """Keep the step count in device memory: every update first advances it on the stream
        and the kernel reads it — so a captured HIP graph replays with the right bias
        correction. ``t`` stays a host mirror (advance it per replay)."""
        if self.t_dev is None:
            self.t_dev = torch.full((1,), self.t, dtype=torch.int32, device=self.p.device)

    @torch.no_grad()
    def step(self, grad: torch.Tensor, working_bf16: Optional[torch.Tensor] = None,
             grad_scale: float = 1.0) -> None:
        self.t += 1
        b1, b2 = self.betas
        if grad.numel() != self.p.numel():
            raise ValueError("grad / master size mismatch")
        if use_hip(self.p, grad) and self.t_dev is not None:
            self.t_dev.add_(1)
            check(_lib.lib().dlbb_adamw_devstep(
                self.p.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), grad.data_ptr(),
                dt(grad), _lib.ptr(working_bf16), self.p.numel(), self.lr, b1, b2, self.eps,
                self.wd, self.t_dev.data_ptr(), float(grad_scale), _lib.stream(self.p.device)),
                "adamw_devstep")
            return
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
