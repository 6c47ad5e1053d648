"""MFMA bf16 GEMM with fused epilogues (``csrc/gemm.hip``).

``linear(x, w, bias, act, residual, out_dtype)`` computes ``act(x @ w.T + bias) + residual``
with ``w`` stored ``[out_features, in_features]`` (K-contiguous, the MFMA-native layout).
Reference call sites: ``models.py:47`` (column-parallel) and ``models.py:81`` (row-parallel).

Shape contract of the HIP kernel: ``K % 64 == 0``, 16-byte aligned rows; M and N arbitrary.
Shapes outside the contract are routed to ``torch.matmul`` (hipBLASLt) — a plain library GEMM —
and counted in :data:`FALLBACKS` so benchmarks can report it.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, use_hip

EPI_BIAS, EPI_GELU_ERF, EPI_GELU_TANH, EPI_RESIDUAL = 1, 2, 4, 8
ACTS = {None: 0, "none": 0, "gelu": EPI_GELU_ERF, "gelu_erf": EPI_GELU_ERF,
        "gelu_tanh": EPI_GELU_TANH}

FALLBACKS = {"count": 0}


def hip_supported(x2: torch.Tensor, w: torch.Tensor) -> bool:
    K = x2.shape[1]
    return (x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and K % 64 == 0
            and x2.stride(1) == 1 and w.stride(1) == 1 and x2.stride(0) % 8 == 0
            and w.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def _torch_linear(x2, w, bias, act, residual, out_dtype, preact):
    y = torch.matmul(x2.float(), w.float().t()) if x2.device.type == "cpu" else x2 @ w.t()
    y = y.float()
    if bias is not None:
        y = y + bias.float()
    if preact is not None:
        preact.copy_(y.to(preact.dtype))
    if act in ("gelu", "gelu_erf"):
        y = F.gelu(y)
    elif act == "gelu_tanh":
        y = F.gelu(y, approximate="tanh")
    if residual is not None:
        y = y + residual.reshape(y.shape).float()
    return y.to(out_dtype)


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           act: Optional[str] = None, residual: Optional[torch.Tensor] = None,
           out_dtype: Optional[torch.dtype] = None, out: Optional[torch.Tensor] = None,
           preact: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``act(x @ w.T + bias) + residual``; x ``[..., K]``, w ``[N, K]``; returns ``[..., N]``."""
    lead = x.shape[:-1]
    K = x.shape[-1]
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"linear: x[..., {K}] vs w{tuple(w.shape)}")
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    out_dtype = out_dtype or x.dtype
    if act not in ACTS:
        raise ValueError(f"unknown activation {act!r}")
    if use_hip(x, w):
        if not hip_supported(x2, w):
            FALLBACKS["count"] += 1
            y = _torch_linear(x2, w, bias, act, residual, out_dtype, preact)
            return y.reshape(*lead, N) if out is None else out.copy_(y.reshape(out.shape))
        if out is None:
            out = torch.empty(*lead, N, dtype=out_dtype, device=x.device)
        if out.dtype not in (torch.bfloat16, torch.float32) or not out.is_contiguous():
            raise ValueError("linear: out must be contiguous bf16/fp32")
        epi = ACTS[act]
        if bias is not None:
            epi |= EPI_BIAS
            bias = bias.contiguous()
        r2 = None
        if residual is not None:
            epi |= EPI_RESIDUAL
            r2 = residual.reshape(M, N)
            if r2.stride(1) != 1 or r2.dtype != torch.bfloat16:
                r2 = r2.contiguous().to(torch.bfloat16)
        check(_lib.lib().dlbb_gemm_bf16_nt(
            x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), N, M, N, K,
            _lib.ptr(bias), _lib.ptr(r2), r2.stride(0) if r2 is not None else 0,
            _lib.ptr(preact), epi, 1 if out.dtype == torch.float32 else 0,
            _lib.stream(x.device)), "gemm_bf16_nt")
        return out
    y = _torch_linear(x2, w, bias, act, residual, out_dtype, preact)
    return y.reshape(*lead, N) if out is None else out.copy_(y.reshape(out.shape))
