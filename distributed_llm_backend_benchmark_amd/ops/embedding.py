"""Token + position embedding with in-place gradient accumulation (``csrc/embedding.hip``).

``embedding(idx, wte, wpe)`` = ``wte[idx] + wpe[:T]`` for ``idx [B, T]``. On the GPU the forward
is one fused gather+add kernel; the backward sorts the B*T token ids once (stable, so the
per-row summation order is fixed) and one kernel accumulates every dX row into its vocabulary
row and every position's batch sum into ``wpe`` — straight into the parameters' ``.grad`` when
they are gradient sinks (the trainer's flat bucket views; see :mod:`.linear_fn`), otherwise into
zero-initialised gradient tensors that are returned to autograd.

Tied embeddings (GPT-2: ``wte`` is also the LM head) are gradient sinks with
``_dlbb_sink_uses = 2``: each use accumulates into ``.grad`` and the sink callback fires after
the last one (:func:`.linear_fn.sink_used`).
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, use_hip


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe):
        B, T = idx.shape
        V, C = wte.shape
        ids = idx.reshape(-1).contiguous().to(torch.int64)
        out = torch.empty(B, T, C, dtype=wte.dtype, device=wte.device)
        check(_lib.lib().dlbb_embedding_fwd(ids.data_ptr(), wte.data_ptr(), wpe.data_ptr(),
                                            out.data_ptr(), B * T, T, C, V,
                                            _lib.stream(wte.device)), "embedding_fwd")
        ctx.save_for_backward(ids)
        ctx.params = (wte, wpe)
        ctx.T = T
        return out

    @staticmethod
    def backward(ctx, dx):
        from .linear_fn import _sink, sink_used

        (ids,) = ctx.saved_tensors
        wte, wpe = ctx.params
        T = ctx.T
        N = ids.numel()
        C = wte.shape[1]
        d2 = dx.reshape(N, C)
        if not d2.is_contiguous() or d2.dtype != torch.bfloat16:
            d2 = d2.contiguous().to(torch.bfloat16)
        need_e, need_p = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        sink_e = _sink(wte) if need_e else None
        sink_p = _sink(wpe) if need_p else None
        # accumulate in place into the sink buffers; otherwise into fresh fp32 zeros
        ge = gp = None
        if need_e:
            ge = wte.grad if sink_e is not None else torch.zeros(wte.shape, dtype=torch.float32,
                                                                  device=wte.device)
        if need_p:
            gp = wpe.grad if sink_p is not None else torch.zeros(wpe.shape, dtype=torch.float32,
                                                                  device=wpe.device)
        # one kernel handles both; it takes one gradient dtype: when the two differ, run twice
        groups = [(ge, gp)] if (ge is None or gp is None or ge.dtype == gp.dtype) \
            else [(ge, None), (None, gp)]
        sorted_ids = order = None
        if ge is not None:
            sorted_ids, order = sort_ids(ids, wte.shape[0])
        if sink_e is not None and getattr(wte, "_dlbb_grad_event", None) is not None:
            # the tied LM head's weight gradient may still be accumulating into the same buffer
            # on a weight-gradient side stream (ops/linear_fn.py): order after that enqueue (not
            # after the whole side stream, whose later weight gradients may overlap this kernel)
            torch.cuda.current_stream(d2.device).wait_event(wte._dlbb_grad_event)
        for e, p in groups:
            g_dt = (e if e is not None else p).dtype
            check(_lib.lib().dlbb_embedding_bwd(
                _lib.ptr(sorted_ids) if e is not None else None,
                _lib.ptr(order) if e is not None else None, d2.data_ptr(), _lib.ptr(e),
                _lib.ptr(p), _lib._DT[g_dt], N, T, C, wte.shape[0],
                _lib.stream(d2.device)), "embedding_bwd")
        out_e = out_p = None
        if need_e:
            if sink_e is not None:
                sink_used(wte)
            else:
                out_e = ge.to(wte.dtype)
        if need_p:
            if sink_p is not None:
                sink_used(wpe)
            else:
                out_p = gp.to(wpe.dtype)
        return None, out_e, out_p   # out_p: full wpe shape, rows >= T zero


def sort_ids(ids: torch.Tensor, vocab: int):
    """Stable ascending sort of int64 token ids -> (sorted ids, positions), both int64. One
    workgroup's block radix sort (``dlbb_sort_ids``: at most 16384 ids, vocabulary < 2^18 —
    pure kernel work, no device memcpy, so a captured step stays kernel-only); the library sort
    beyond that."""
    n = ids.numel()
    if ids.is_cuda and ids.dtype == torch.int64 and ids.is_contiguous() and n <= 16384 \
            and vocab <= (1 << 18) and os.environ.get("DLBB_SORT_IDS", "hip") != "torch":
        s = torch.empty_like(ids)
        o = torch.empty_like(ids)
        check(_lib.lib().dlbb_sort_ids(ids.data_ptr(), s.data_ptr(), o.data_ptr(), n, int(vocab),
                                       _lib.stream(ids.device)), "sort_ids")
        return s, o
    return torch.sort(ids, stable=True)


def embedding(idx: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor) -> torch.Tensor:
    """``wte[idx] + wpe[:T]`` for token ids ``idx [B, T]`` (GPT-2 input embedding)."""
    B, T = idx.shape
    C = wte.shape[1]
    if (use_hip(wte, wpe) and wte.dtype == torch.bfloat16 and wpe.dtype == torch.bfloat16
            and C % 8 == 0 and wte.is_contiguous() and wpe.is_contiguous()
            and wte.data_ptr() % 16 == 0 and wpe.data_ptr() % 16 == 0 and wpe.shape[0] >= T):
        return _EmbeddingFn.apply(idx, wte, wpe)
    return F.embedding(idx, wte) + wpe[:T]
