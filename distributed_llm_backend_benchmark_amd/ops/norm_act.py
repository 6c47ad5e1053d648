"""Fused residual+LayerNorm and bias+GELU with autograd (``csrc/layernorm.hip``,
``csrc/gelu.hip``).

Reference ops: ``nn.LayerNorm`` (``models.py:122,135,222``), residual adds
(``models.py:173,188``), ``F.gelu`` (``models.py:182``).
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, dt, use_hip

_LN_BWD_COLS = {256, 512, 768, 1024, 1536, 2048, 3072, 4096}
LN_FALLBACKS = {"count": 0}   # backward calls at widths without a fused-kernel instantiation


def _ln_bwd_reference(dy2, hin, weight, mean, rstd, dh2, dw, db, accumulate: bool):
    """LayerNorm backward in fp32 torch ops (the fused kernel's math): returns dx (+ dh) in the
    activation dtype and writes / accumulates dγ, dβ into ``dw`` / ``db``."""
    xhat = (hin.float() - mean[:, None]) * rstd[:, None]
    g = dy2.float()
    dxhat = g * weight.float()
    dx = rstd[:, None] * (dxhat - dxhat.mean(1, keepdim=True)
                          - xhat * (dxhat * xhat).mean(1, keepdim=True))
    if dh2 is not None:
        dx = dx + dh2.float()
    gw = (g * xhat).sum(0)
    if accumulate:
        dw.add_(gw.to(dw.dtype))
    else:
        dw.copy_(gw)
    if db is not None:
        gb = g.sum(0)
        if accumulate:
            db.add_(gb.to(db.dtype))
        else:
            db.copy_(gb)
    return dx.to(hin.dtype)


def _ln_fwd_hip(x2, r2, weight, bias, eps, need_stats: bool):
    rows, cols = x2.shape
    y = torch.empty_like(x2)
    h = torch.empty_like(x2) if r2 is not None else None
    mean = torch.empty(rows, dtype=torch.float32, device=x2.device) if need_stats else None
    rstd = torch.empty(rows, dtype=torch.float32, device=x2.device) if need_stats else None
    check(_lib.lib().dlbb_layernorm_fwd(
        x2.data_ptr(), _lib.ptr(r2), weight.data_ptr(), _lib.ptr(bias), dt(weight), y.data_ptr(),
        _lib.ptr(h), _lib.ptr(mean), _lib.ptr(rstd), rows, cols, float(eps),
        _lib.stream(x2.device)), "layernorm_fwd")
    return y, h, mean, rstd


class _FusedAddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps):
        shape = x.shape
        cols = shape[-1]
        x2 = x.reshape(-1, cols).contiguous()
        r2 = residual.reshape(-1, cols).contiguous() if residual is not None else None
        y, h, mean, rstd = _ln_fwd_hip(x2, r2, weight, bias, eps, True)
        hin = h if h is not None else x2
        ctx.save_for_backward(hin, weight, mean, rstd)
        ctx.has_res = residual is not None
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)       # leaf parameters: only read for their grad sinks
        ctx.shape = shape
        if h is not None:
            return y.view(shape), h.view(shape)
        return y.view(shape), None

    @staticmethod
    def backward(ctx, dy, dh):
        hin, weight, mean, rstd = ctx.saved_tensors
        rows, cols = hin.shape
        dy2 = dy.reshape(rows, cols).contiguous()
        dh2 = dh.reshape(rows, cols).contiguous() if (dh is not None and ctx.has_res) else None
        # gradient sinks (ops.linear_fn): dγ/dβ accumulate straight into the trainer's views
        from .linear_fn import _sink, sink_fresh, sink_used

        w_p, b_p = ctx.params
        w_sink, b_sink = _sink(w_p), (_sink(b_p) if ctx.has_bias else None)
        direct = w_sink is not None and (not ctx.has_bias or b_sink is not None)
        dw = w_p.grad if direct else torch.empty_like(weight)
        db = (b_p.grad if direct else torch.empty_like(weight)) if ctx.has_bias else None
        accumulate = direct and not (sink_fresh(w_p) and (not ctx.has_bias or sink_fresh(b_p)))
        if cols in _LN_BWD_COLS:
            dx = torch.empty_like(hin)
            grid = _lib.lib().dlbb_layernorm_bwd_grid(rows)
            ws = torch.empty((2 if ctx.has_bias else 1) * grid * cols, dtype=torch.float32,
                             device=hin.device)
            check(_lib.lib().dlbb_layernorm_bwd(
                dy2.data_ptr(), hin.data_ptr(), weight.data_ptr(), dt(weight), mean.data_ptr(),
                rstd.data_ptr(), _lib.ptr(dh2), dx.data_ptr(), ws.data_ptr(), dw.data_ptr(),
                _lib.ptr(db), rows, cols, int(accumulate), _lib.stream(hin.device)),
                "layernorm_bwd")
        else:
            # widths the fused kernel has no instantiation for (cols not a listed multiple of
            # 256, e.g. toy models): the same math in fp32 torch ops, counted in LN_FALLBACKS
            LN_FALLBACKS["count"] += 1
            dx = _ln_bwd_reference(dy2, hin, weight, mean, rstd, dh2, dw, db, accumulate)
        dxv = dx.view(ctx.shape)
        if direct:
            sink_used(w_p)
            if ctx.has_bias:
                sink_used(b_p)
            return dxv, (dxv if ctx.has_res else None), None, None, None
        return dxv, (dxv if ctx.has_res else None), dw, db, None


def layernorm(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
              eps: float = 1e-5, residual: Optional[torch.Tensor] = None
              ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Returns ``(LN(h), h)`` with ``h = x + residual`` (or ``(LN(x), None)``)."""
    if use_hip(x, weight):
        if x.dtype != torch.bfloat16:
            raise _lib.KernelError("fused LayerNorm takes bf16 activations")
        return _FusedAddLayerNorm.apply(x, residual, weight, bias, eps)
    h = x + residual if residual is not None else None
    src = h if h is not None else x
    y = F.layer_norm(src.float(), (x.shape[-1],), weight.float(),
                     bias.float() if bias is not None else None, eps).to(x.dtype)
    return y, h


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, approx: int):
        cols = x.shape[-1]
        x2 = x.reshape(-1, cols).contiguous()
        y = torch.empty_like(x2)
        check(_lib.lib().dlbb_bias_gelu_fwd(x2.data_ptr(), _lib.ptr(bias), y.data_ptr(),
                                            x2.shape[0], cols, approx, _lib.stream(x.device)),
              "bias_gelu_fwd")
        ctx.save_for_backward(x2, bias)
        ctx.approx = approx
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, bias = ctx.saved_tensors
        rows, cols = x2.shape
        dy2 = dy.reshape(rows, cols).contiguous()
        dx = torch.empty_like(x2)
        ws = torch.zeros(cols, dtype=torch.float32, device=x2.device) if bias is not None else None
        check(_lib.lib().dlbb_bias_gelu_bwd(dy2.data_ptr(), x2.data_ptr(), _lib.ptr(bias),
                                            dx.data_ptr(), _lib.ptr(ws), rows, cols, ctx.approx,
                                            _lib.stream(x2.device)), "bias_gelu_bwd")
        db = ws.to(bias.dtype) if bias is not None else None
        return dx.view(ctx.shape), db, None


def bias_gelu(x: torch.Tensor, bias: Optional[torch.Tensor] = None,
              approximate: str = "none") -> torch.Tensor:
    """``gelu(x + bias)``; ``approximate`` = ``"none"`` (erf, reference default) | ``"tanh"``."""
    approx = 1 if approximate == "tanh" else 0
    if use_hip(x):
        if x.dtype != torch.bfloat16 or x.shape[-1] % 8:
            raise _lib.KernelError("bias_gelu takes bf16 with last dim % 8 == 0")
        return _BiasGelu.apply(x, bias, approx)
    u = x.float() + (bias.float() if bias is not None else 0.0)
    return F.gelu(u, approximate=approximate).to(x.dtype)
