"""Causal self-attention on the fused QKV activation (``csrc/attention.hip``).

``causal_attention(qkv, n_head)`` takes a fused ``[B, T, 3C]`` QKV GEMM output (GPT-2's, or a
tensor-parallel rank's shard, models/tp_transformer.py) and returns ``[B, T, C]`` (heads
interleaved, ready for the projection GEMM). The forward is our gfx950 flash kernel (head dim 64
or 128); it reads Q/K/V straight out of ``qkv`` — no unbind/transpose copies — and emits the
per-row log-sum-exp. The backward (head dim 64) is ours too (a query-block kernel for dQ that
also writes the row constants, then a key-block kernel for dK/dV, no atomics), writing the fused
``[B, T, 3C]`` gradient directly. At head dim 128 the backward is the stack's flash backward on
our forward's O / LSE (``attn_bwd_library``: same natural-log ``[B, H, T]`` convention; no
training path here uses it — the TP model is forward only).

Other head dims, CPU tensors and ``DLBB_KERNELS=torch`` use ``F.scaled_dot_product_attention``.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, use_hip


def _views(qkv: torch.Tensor, n_head: int):
    B, T, C3 = qkv.shape
    C = C3 // 3
    q, k, v = qkv.view(B, T, 3, n_head, C // n_head).permute(2, 0, 3, 1, 4).unbind(0)
    return q, k, v


def _torch_attention(qkv: torch.Tensor, n_head: int) -> torch.Tensor:
    B, T, C3 = qkv.shape
    q, k, v = _views(qkv, n_head)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    return y.transpose(1, 2).reshape(B, T, C3 // 3)


HEAD_DIMS = (64, 128)


def hip_supported(qkv: torch.Tensor, n_head: int) -> bool:
    if qkv.dim() != 3 or qkv.dtype != torch.bfloat16 or not qkv.is_contiguous():
        return False
    C = qkv.shape[2] // 3
    return qkv.shape[2] % 3 == 0 and C % n_head == 0 and C // n_head in HEAD_DIMS


def attn_fwd(qkv: torch.Tensor, n_head: int):
    """Raw forward: (out [B, T, C] bf16, lse [B, H, T] fp32)."""
    B, T, C3 = qkv.shape
    C = C3 // 3
    D = C // n_head
    out = torch.empty(B, T, C, dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty(B, n_head, T, dtype=torch.float32, device=qkv.device)
    check(_lib.lib().dlbb_attn_fwd(qkv.data_ptr(), C3, out.data_ptr(), C, lse.data_ptr(), B, T,
                                   n_head, D, 1.0 / math.sqrt(D), _lib.stream(qkv.device)),
          "attn_fwd")
    return out, lse


class _CausalAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, n_head):
        out, lse = attn_fwd(qkv, n_head)
        ctx.save_for_backward(qkv, out, lse)
        ctx.n_head = n_head
        return out

    @staticmethod
    def backward(ctx, gout):
        qkv, out, lse = ctx.saved_tensors
        if (qkv.shape[2] // 3) // ctx.n_head != 64:
            return attn_bwd_library(qkv, out, lse, gout.contiguous(), ctx.n_head), None
        return attn_bwd(qkv, out, lse, gout, ctx.n_head), None


def attn_bwd(qkv: torch.Tensor, out: torch.Tensor, lse: torch.Tensor, gout: torch.Tensor,
             n_head: int) -> torch.Tensor:
    """Raw backward: dQKV [B, T, 3C] (dkdv + dq kernels, no atomics)."""
    B, T, C3 = qkv.shape
    C = C3 // 3
    D = C // n_head
    gout = gout.contiguous()
    dqkv = torch.empty_like(qkv)
    # workspace: -rowsum(dO * O) and -LSE * sqrt(D), [2, B, H, T] (csrc/attention.hip)
    delta = torch.empty(2, B, n_head, T, dtype=torch.float32, device=qkv.device)
    check(_lib.lib().dlbb_attn_bwd(qkv.data_ptr(), C3, out.data_ptr(), gout.data_ptr(), C,
                                   lse.data_ptr(), delta.data_ptr(), dqkv.data_ptr(), B, T, n_head,
                                   D, 1.0 / math.sqrt(D), _lib.stream(qkv.device)), "attn_bwd")
    return dqkv


def attn_bwd_library(qkv, out, lse, gout, n_head: int) -> torch.Tensor:
    """The stack's flash backward on our forward's (O, LSE), dQ/dK/dV packed into [B, T, 3C]
    (head dim 128, and the A/B baseline for :func:`attn_bwd`)."""
    B, T, C3 = qkv.shape
    C = C3 // 3
    D = C // n_head
    q, k, v = _views(qkv, n_head)
    o4 = out.view(B, T, n_head, D).transpose(1, 2)
    g4 = gout.reshape(B, T, n_head, D).transpose(1, 2)
    seed = torch.zeros((), dtype=torch.int64, device=qkv.device)
    dq, dk, dv = torch.ops.aten._scaled_dot_product_flash_attention_backward(
        g4, q, k, v, o4, lse, None, None, T, T, 0.0, True, seed, seed, scale=1.0 / math.sqrt(D))
    dqkv = torch.empty_like(qkv)
    lib = _lib.lib()
    st = _lib.stream(qkv.device)
    for j, g in enumerate((dq, dk, dv)):
        g2 = g.transpose(1, 2)
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        check(lib.dlbb_pack_rows(g2.data_ptr(), _lib.DT_BF16, C, dqkv.data_ptr() + j * C * 2,
                                 _lib.DT_BF16, C3, B * T, C, st), "pack_rows(dqkv)")
    return dqkv


def causal_attention(qkv: torch.Tensor, n_head: int) -> torch.Tensor:
    """Causal multi-head self-attention of a fused ``[B, T, 3C]`` QKV tensor -> ``[B, T, C]``."""
    if use_hip(qkv) and hip_supported(qkv, n_head):
        return _CausalAttention.apply(qkv, n_head)
    return _torch_attention(qkv, n_head)
