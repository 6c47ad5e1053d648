"""Fused softmax cross-entropy on bf16 logits (``csrc/xent.hip``), mean reduction over the
non-ignored rows (``ignore_index`` = any negative target).

``linear_cross_entropy(x, w, target)`` fuses the LM head with the loss: the forward GEMM writes
the logits, ONE kernel pass turns them in place into ``dlogits / count`` and per-row losses
(the loss forward and backward share a single read of the logits), and the backward only
runs the two GEMMs, with the upstream gradient applied to their small outputs / inputs."""

from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from . import gemm as _gemm
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


class _LinearXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, target):
        from .gemm import linear

        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        V = w.shape[0]
        logits = linear(x2, w)                          # [rows, V] bf16 (autotuned GEMM)
        t = target.reshape(-1).contiguous().to(torch.int64)
        rows = x2.shape[0]
        loss = torch.empty(rows + 2, dtype=torch.float32, device=x2.device)
        inv, out = loss[rows:rows + 1], loss[rows + 1:]  # 1 / count and the mean, same buffer
        st = _lib.stream(x2.device)
        check(_lib.lib().dlbb_xent_count_inv(t.data_ptr(), rows, inv.data_ptr(), st),
              "xent_count_inv")
        check(_lib.lib().dlbb_xent_fused(logits.data_ptr(), t.data_ptr(), loss.data_ptr(), rows,
                                         V, V, inv.data_ptr(), st), "xent_fused")
        check(_lib.lib().dlbb_xent_loss_mean(loss.data_ptr(), rows, inv.data_ptr(),
                                             out.data_ptr(), st), "xent_loss_mean")
        ctx.save_for_backward(x2, w, logits)            # logits now hold dlogits / count
        ctx.shape = x.shape
        ctx.weight = w                                  # leaf parameter: read for its grad sink
        return out.reshape(())

    @staticmethod
    def backward(ctx, g):
        from .gemm import wgrad

        from .linear_fn import _sink, sink_fresh, sink_used

        x2, w, dl = ctx.saved_tensors
        # the caller may mark the upstream gradient as exactly 1 (mark_unit_upstream: this output
        # IS the loss passed to .backward()): then no scaling passes over dX and X (2 x 25 MB on
        # the GPT-2 step's critical path)
        unit = getattr(ctx, "dlbb_unit_upstream", False)
        gb = None if unit else g.to(dl.dtype)
        xs = x2 if unit else x2 * gb
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = _gemm.dgrad(dl, w)
            if not unit:
                dx.mul_(gb)
            dx = dx.view(ctx.shape)
        if ctx.needs_input_grad[1]:
            if _sink(ctx.weight) is not None:
                # gradient sink (e.g. the tied embedding): accumulate into .grad in the GEMM —
                # or store, when this is the first write since zero_grad (the LM head is the
                # first op of the backward: a beta = 0 GEMM, no read of the 77 MB buffer)
                wgrad(dl, xs, out=ctx.weight.grad, accumulate=not sink_fresh(ctx.weight))
                sink_used(ctx.weight)
            else:
                dw = wgrad(dl, xs)
        return dx, dw, None


def mark_unit_upstream(loss: torch.Tensor) -> bool:
    """Declare that ``loss`` itself is what ``.backward()`` is called on (upstream gradient
    exactly 1): if it is the output of the fused LM head + loss, its backward then skips the
    upstream-gradient scaling passes. Returns whether it applied (trainers call it on the loss
    their model returned)."""
    fn = getattr(loss, "grad_fn", None)
    if fn is None or type(fn).__name__ != "_LinearXentFnBackward" or loss.dim() != 0:
        return False
    fn.dlbb_unit_upstream = True
    return True


def linear_cross_entropy(x: torch.Tensor, w: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """``cross_entropy(x @ w.T, target)`` (mean over rows with target >= 0), LM-head fused."""
    from .gemm import hip_supported

    V = w.shape[0]
    if (use_hip(x, w) and x.dtype == torch.bfloat16 and V % 8 == 0 and V <= 8 * 512 * 16
            and hip_supported(x.reshape(-1, x.shape[-1]), w)):
        return _LinearXentFn.apply(x, w, target)
    from .linear_fn import linear_train

    return cross_entropy(linear_train(x, w), target)


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    if use_hip(logits) and logits.dtype == torch.bfloat16 and logits.shape[-1] % 8 == 0:
        return _XentFn.apply(logits, target)
    V = logits.shape[-1]
    return F.cross_entropy(logits.float().reshape(-1, V), target.reshape(-1), ignore_index=-100)
