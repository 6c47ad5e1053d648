"""Fused softmax cross-entropy on bf16 logits (``csrc/xent.hip``), mean reduction over the
non-ignored rows (``ignore_index`` = any negative target)."""

from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, use_hip


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        V = logits.shape[-1]
        x2 = logits.reshape(-1, V).contiguous()
        t = target.reshape(-1).contiguous().to(torch.int64)
        rows = x2.shape[0]
        loss = torch.empty(rows, dtype=torch.float32, device=x2.device)
        lse = torch.empty(rows, dtype=torch.float32, device=x2.device)
        check(_lib.lib().dlbb_xent_fwd(x2.data_ptr(), t.data_ptr(), loss.data_ptr(),
                                       lse.data_ptr(), rows, V, x2.stride(0),
                                       _lib.stream(x2.device)), "xent_fwd")
        count = (t >= 0).sum().clamp_min(1).float()
        ctx.save_for_backward(x2, t, lse, count)
        ctx.shape = logits.shape
        return loss.sum() / count

    @staticmethod
    def backward(ctx, g):
        x2, t, lse, count = ctx.saved_tensors
        rows, V = x2.shape
        dx = torch.empty(rows, V, dtype=x2.dtype, device=x2.device)
        scale = (g.float() / count).reshape(1).contiguous()   # stays on device: no sync
        check(_lib.lib().dlbb_xent_bwd(x2.data_ptr(), t.data_ptr(), lse.data_ptr(),
                                       dx.data_ptr(), rows, V, V, scale.data_ptr(),
                                       _lib.stream(x2.device)), "xent_bwd")
        return dx.view(ctx.shape), None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    if use_hip(logits) and logits.dtype == torch.bfloat16 and logits.shape[-1] % 8 == 0:
        return _XentFn.apply(logits, target)
    V = logits.shape[-1]
    return F.cross_entropy(logits.float().reshape(-1, V), target.reshape(-1), ignore_index=-100)
