"""Trainable linear: MFMA forward with fused bias/GELU epilogue, MFMA backward.

Forward: ``y = act(x @ W^T + b)`` through the hand-written MFMA kernel (``csrc/gemm.hip``);
with an activation the epilogue also stores the pre-activation ``u`` (needed by the GELU
backward). Backward: ``dU = dY * act'(u)`` and ``db = colsum(dU)`` in one pass of the bias-GELU
backward kernel (``csrc/gelu.hip``); ``dX = dU @ W`` through :func:`.gemm.dgrad` (the NN
transposed-read MFMA kernel or the library, per-shape autotune); ``dW = dU^T @ X`` through
:func:`.gemm.wgrad` (our split-K transposed-read MFMA kernel or the library, per-shape
autotune), which also produces ``db = colsum(dU)`` (an all-ones MFMA operand in the same
kernel). :func:`mlp_train` fuses a whole MLP (linear -> GELU -> linear) so the GELU backward
runs in the dgrad GEMM's epilogue instead of its own pass.

Gradient sinks: a trainer that keeps ``.grad`` as views of a flat bucket buffer can mark a
parameter with ``_dlbb_grad_sink = callback`` (only for parameters used ONCE per forward — the
model opts in with ``_dlbb_single_use``). The backward then accumulates dW / db straight into
``param.grad`` inside the weight-gradient kernel's reduce pass, calls ``callback(param)`` and
returns no gradient for it — no separate gradient tensor and no AccumulateGrad add kernel.
With ``_dlbb_grad_stream`` also set, that weight-gradient GEMM runs on the given side stream.
"""

from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from . import gemm as _gemm
from ._lib import check, use_hip
from .gemm import hip_supported, linear as _linear, wgrad

_APPROX = {"gelu": 0, "gelu_erf": 0, "gelu_tanh": 1}


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if x2.stride(-1) != 1 or x2.stride(0) % 8:
            x2 = x2.contiguous()
        M, N = x2.shape[0], w.shape[0]
        u = None
        if act is not None:
            u = torch.empty(M, N, dtype=x.dtype, device=x.device)
        y = _linear(x2, w, bias=b, act=act, preact=u)
        ctx.save_for_backward(x2, w, u)
        ctx.has_bias = b is not None
        ctx.weight, ctx.bias = w, b   # leaf parameters: only read for their grad sinks
        ctx.act = act
        ctx.lead = x.shape[:-1]
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, u = ctx.saved_tensors
        M, K = x2.shape
        N = w.shape[0]
        dy2 = dy.reshape(M, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        fuse_db = want_db and ctx.needs_input_grad[1]   # db rides on the wgrad kernels
        db = None
        if ctx.act is not None:
            du = torch.empty_like(u)
            ws = (torch.zeros(N, dtype=torch.float32, device=u.device)
                  if want_db and not fuse_db else None)
            check(_lib.lib().dlbb_bias_gelu_bwd(dy2.data_ptr(), u.data_ptr(), None, du.data_ptr(),
                                                _lib.ptr(ws), M, N, _APPROX[ctx.act],
                                                _lib.stream(u.device)), "bias_gelu_bwd")
            if ws is not None:
                db = ws.to(w.dtype)
        else:
            du = dy2
            if want_db and not fuse_db:
                db = du.sum(0, dtype=torch.float32).to(w.dtype)
        dx = _gemm.dgrad(du, w) if ctx.needs_input_grad[0] else None
        dw, db = _weight_grads(ctx.weight, ctx.bias, du, x2, ctx.needs_input_grad[1], want_db,
                               db)
        if dx is not None:
            dx = dx.view(*ctx.lead, K)
        return dx, dw, db, None


def _weight_grads(weight, bias, du, x2, need_w: bool, want_db: bool, db=None):
    """``dW = du^T @ x2`` and ``db = colsum(du)`` (fused into the weight-gradient kernels when
    both are wanted). Into the parameters' gradient sinks when they take it (then returns
    ``(None, None)`` — autograd gets no gradient tensor), else as fresh tensors. ``db``: a bias
    gradient already computed elsewhere (used when dW is not wanted)."""
    fuse_db = want_db and need_w
    w_sink = _sink(weight) if need_w else None
    b_sink = _sink(bias) if fuse_db else None
    if w_sink is not None and (not want_db or b_sink is not None):
        # store instead of accumulate while the buffers are still this step's zeros
        acc = not (sink_fresh(weight) and (not want_db or sink_fresh(bias)))
        side = getattr(weight, "_dlbb_grad_stream", None)
        if side is not None:
            # dW is off the backward's critical path: run it on the trainer's side stream
            # so it overlaps the next layer's dgrad / memory-bound kernels; the trainer
            # orders its bucket reductions and the optimizer after that stream
            from ..parallel.streams import fork

            fork(side)                      # no system-scope fence (parallel/streams.py)
            with torch.cuda.stream(side):
                wgrad(du, x2, out=weight.grad, accumulate=acc,
                      bias_out=bias.grad if want_db else None)
            du.record_stream(side)
            x2.record_stream(side)
            if getattr(weight, "_dlbb_sink_uses", 1) > 1:
                # a multi-use sink (tied LM head / embedding): its other uses accumulate into the
                # same buffer from other streams and wait for THIS enqueue only (ops/embedding.py)
                ev = getattr(weight, "_dlbb_grad_event", None)
                if ev is None:
                    ev = weight._dlbb_grad_event = torch.cuda.Event()
                ev.record(side)
        else:
            wgrad(du, x2, out=weight.grad, accumulate=acc,
                  bias_out=bias.grad if want_db else None)
        sink_used(weight)
        if want_db:
            sink_used(bias)
        return None, None
    dw = None
    if need_w:
        N, K = du.shape[1], x2.shape[1]
        dw = torch.empty(N, K, dtype=du.dtype, device=du.device)
        if fuse_db:
            db = torch.empty(N, dtype=du.dtype, device=du.device)
        wgrad(du, x2, out=dw, bias_out=db if fuse_db else None)
    elif want_db and db is None:
        db = du.sum(0, dtype=torch.float32)
    if db is not None and db.dtype != weight.dtype:
        db = db.to(weight.dtype)
    return dw, (db if want_db else None)


class _MLPFn(torch.autograd.Function):
    """``act(x @ W1^T + b1) @ W2^T + b2`` as one autograd op, so the GELU backward runs in the
    epilogue of the GEMM that produces its input gradient: ``du = (dY @ W2) * act'(u)`` from
    the NN dgrad kernel (``u`` = the pre-activation stored by the first GEMM's epilogue) instead
    of a dgrad GEMM writing ``dg`` plus a separate bias-GELU backward pass reading it back."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, act):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if x2.stride(-1) != 1 or x2.stride(0) % 8:
            x2 = x2.contiguous()
        M, N1 = x2.shape[0], w1.shape[0]
        u = torch.empty(M, N1, dtype=x.dtype, device=x.device)
        g = _linear(x2, w1, bias=b1, act=act, preact=u)
        y = _linear(g, w2, bias=b2)
        ctx.save_for_backward(x2, w1, u, g, w2)
        ctx.params = (w1, b1, w2, b2)
        ctx.act = act
        ctx.lead = x.shape[:-1]
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w1, u, g, w2 = ctx.saved_tensors
        p_w1, p_b1, p_w2, p_b2 = ctx.params
        M, K = x2.shape
        dy2 = dy.reshape(M, w2.shape[0])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        nig = ctx.needs_input_grad
        need_u = nig[0] or nig[1] or nig[2]
        du = _gemm.dgrad(dy2, w2, dgelu=(u, ctx.act)) if need_u else None
        dw2, db2 = _weight_grads(p_w2, p_b2, dy2, g, nig[3], p_b2 is not None and nig[4])
        dx = _gemm.dgrad(du, w1) if nig[0] else None
        dw1 = db1 = None
        if du is not None:
            dw1, db1 = _weight_grads(p_w1, p_b1, du, x2, nig[1], p_b1 is not None and nig[2])
        if dx is not None:
            dx = dx.view(*ctx.lead, K)
        return dx, dw1, db1, dw2, db2, None


def _sink(p: Optional[torch.Tensor]):
    """The parameter's gradient-sink callback if its .grad can take an in-kernel accumulate."""
    cb = getattr(p, "_dlbb_grad_sink", None) if p is not None else None
    g = p.grad if cb is not None else None
    if g is None or g.dtype != p.dtype or g.shape != p.shape or not g.is_contiguous():
        return None
    return cb


def sink_fresh(p: torch.Tensor) -> bool:
    """True if the sink parameter's ``.grad`` is still the zeros the trainer wrote this step (no
    write since ``zero_grad``): a writer may then store instead of accumulate."""
    return bool(getattr(p, "_dlbb_grad_fresh", False))


def sink_used(p: torch.Tensor) -> None:
    """Record one in-kernel accumulation into a sink parameter's ``.grad``; the sink callback
    fires after the parameter's last use of the step (``_dlbb_sink_uses``, default 1 — e.g. 2
    for a tied embedding / LM-head weight), so the trainer sees the gradient complete."""
    p._dlbb_grad_fresh = False          # the buffer now holds this step's partial gradient
    uses = getattr(p, "_dlbb_sink_uses", 1)
    n = getattr(p, "_dlbb_sink_count", 0) + 1
    if n >= uses:
        p._dlbb_sink_count = 0
        p._dlbb_grad_sink(p)
    else:
        p._dlbb_sink_count = n


def linear_train(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
                 act: Optional[str] = None) -> torch.Tensor:
    """Autograd-aware ``act(x @ w.T + b)``; HIP MFMA forward on GPU tensors."""
    if use_hip(x, w) and hip_supported(x.reshape(-1, x.shape[-1]), w):
        if act is not None and w.shape[0] % 8:
            raise _lib.KernelError("linear_train with activation needs N % 8 == 0")
        return _LinearFn.apply(x, w, b, act)
    y = F.linear(x, w, b)
    if act in ("gelu", "gelu_erf"):
        y = F.gelu(y)
    elif act == "gelu_tanh":
        y = F.gelu(y, approximate="tanh")
    return y


def mlp_train(x: torch.Tensor, w1: torch.Tensor, b1: Optional[torch.Tensor], w2: torch.Tensor,
              b2: Optional[torch.Tensor], act: str = "gelu_tanh") -> torch.Tensor:
    """Autograd-aware ``act(x @ w1.T + b1) @ w2.T + b2`` (a transformer MLP). On GPU the GELU
    backward is fused into the dgrad GEMM's epilogue (:class:`_MLPFn`); elsewhere two
    :func:`linear_train` calls (also with ``DLBB_FUSED_MLP=0``, for A/B)."""
    x2 = x.reshape(-1, x.shape[-1])
    if (use_hip(x, w1) and hip_supported(x2, w1) and w1.shape[0] % 8 == 0
            and os.environ.get("DLBB_FUSED_MLP", "1") != "0"
            and w2.shape[1] == w1.shape[0] and act in _APPROX):
        return _MLPFn.apply(x, w1, b1, w2, b2, act)
    return linear_train(linear_train(x, w1, b1, act=act), w2, b2)
