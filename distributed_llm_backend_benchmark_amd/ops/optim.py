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
             grad_scale: float = 1.0, ranges=None, advance: bool = True) -> None:
        """One AdamW update. ``ranges``: update only these [start, end) element ranges (one
        kernel each; the rest of the step's ranges follow in later calls with
        ``advance=False``, so the step count — and the bias correction — moves once)."""
        if grad.numel() != self.p.numel():
            raise ValueError("grad / master size mismatch")
        if advance:
            self.t += 1
            if self.t_dev is not None and use_hip(self.p, grad):
                self.t_dev.add_(1)
        b1, b2 = self.betas
        n = self.p.numel()
        for a, e in (ranges or [(0, n)]):
            if not 0 <= a <= e <= n:
                raise ValueError(f"AdamW range [{a}, {e}) outside [0, {n})")
            if e == a:
                continue
            p, m, v, g = self.p[a:e], self.m[a:e], self.v[a:e], grad[a:e]
            w = working_bf16[a:e] if working_bf16 is not None else None
            if use_hip(self.p, grad) and self.t_dev is not None:
                check(_lib.lib().dlbb_adamw_devstep(
                    p.data_ptr(), m.data_ptr(), v.data_ptr(), g.data_ptr(), dt(grad),
                    _lib.ptr(w), e - a, self.lr, b1, b2, self.eps, self.wd,
                    self.t_dev.data_ptr(), float(grad_scale), _lib.stream(self.p.device)),
                    "adamw_devstep")
            elif use_hip(self.p, grad):
                check(_lib.lib().dlbb_adamw(
                    p.data_ptr(), m.data_ptr(), v.data_ptr(), g.data_ptr(), dt(grad),
                    _lib.ptr(w), e - a, self.lr, b1, b2, self.eps, self.wd, self.t,
                    float(grad_scale), _lib.stream(self.p.device)), "adamw")
            else:
                gf = g.float() * grad_scale
                m.mul_(b1).add_(gf, alpha=1 - b1)
                v.mul_(b2).addcmul_(gf, gf, value=1 - b2)
                bc1 = 1 - b1 ** self.t
                bc2 = 1 - b2 ** self.t
                denom = (v / bc2).sqrt_().add_(self.eps)
                p.mul_(1 - self.lr * self.wd).addcdiv_(m, denom, value=-self.lr / bc1)
                if w is not None:
                    w.copy_(p.to(w.dtype))
