"""GPT-2 (small by default) for the DDP training microbenchmark (BASELINE config 5: "GPT-2-small
DDP training microbench (models.py path), grad-bucket all-reduce overlapped with backward").

The reference's only training step is a 10→20→5 MLP under DeepSpeed ZeRO-2 (``test/ccl.py:59-117``)
and its transformer is forward-only (``models.py``); this model is the training-side family the
north star asks for, built from the same gfx950 kernels as the TP model:

* residual adds fused into the following LayerNorm (``ops.layernorm(x, residual=h)``),
* QKV / attention-out / MLP / LM-head GEMMs on the MFMA kernel with fused bias and, for c_fc,
  fused tanh-GELU (pre-activation kept for backward),
* causal attention: our gfx950 flash forward on the fused QKV (ops.causal_attention),
* the LM head and its loss as one op (``ops.linear_cross_entropy``): the logits are turned
  into per-row losses and dlogits in place by one fused kernel pass.

All parameters are bf16 working copies (the trainer keeps fp32 masters); vocab is padded to a
multiple of 128 (50257 → 50304) so the tied LM-head GEMM fits the MFMA tiling.
Weights: N(0, 0.02), residual projections scaled by 1/sqrt(2*n_layer) (GPT-2 init).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from ..ops.linear_fn import linear_train, mlp_train


@dataclass
class GPT2Config:
    vocab_size: int = 50304
    block_size: int = 1024
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768


def _param(shape, std, device, gen, dtype=torch.bfloat16):
    t = torch.zeros(*shape, device=device, dtype=torch.float32)
    if std > 0:
        t.normal_(0.0, std, generator=gen)
    return nn.Parameter(t.to(dtype))


class LN(nn.Module):
    def __init__(self, d, device):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d, device=device, dtype=torch.bfloat16))
        self.bias = nn.Parameter(torch.zeros(d, device=device, dtype=torch.bfloat16))
        self.weight._dlbb_single_use = self.bias._dlbb_single_use = True   # see Block

    def forward(self, x, residual=None):
        y, h = ops.layernorm(x, self.weight, self.bias, 1e-5, residual=residual)
        return y, (h if h is not None else x)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config, device, gen):
        super().__init__()
        d = cfg.n_embd
        proj_std = 0.02 / math.sqrt(2 * cfg.n_layer)
        self.n_head = cfg.n_head
        self.ln_1 = LN(d, device)
        self.attn_w = _param((3 * d, d), 0.02, device, gen)
        self.attn_b = _param((3 * d,), 0.0, device, gen)
        self.attn_proj_w = _param((d, d), proj_std, device, gen)
        self.attn_proj_b = _param((d,), 0.0, device, gen)
        self.ln_2 = LN(d, device)
        self.fc_w = _param((4 * d, d), 0.02, device, gen)
        self.fc_b = _param((4 * d,), 0.0, device, gen)
        self.mlp_proj_w = _param((d, 4 * d), proj_std, device, gen)
        self.mlp_proj_b = _param((d,), 0.0, device, gen)
        # used exactly once per forward (by linear_train): a trainer may accumulate their
        # gradients in-kernel into its flat buffer (ops.linear_fn gradient sinks)
        for p in (self.attn_w, self.attn_b, self.attn_proj_w, self.attn_proj_b, self.fc_w,
                  self.fc_b, self.mlp_proj_w, self.mlp_proj_b):
            p._dlbb_single_use = True

    def forward(self, y1, h):
        B, T, C = y1.shape
        qkv = linear_train(y1, self.attn_w, self.attn_b)
        att = ops.causal_attention(qkv, self.n_head)
        a = linear_train(att, self.attn_proj_w, self.attn_proj_b)
        y2, h = self.ln_2(a, residual=h)
        # fc -> GELU -> proj as one op: the GELU backward rides in the proj dgrad's epilogue
        d = mlp_train(y2, self.fc_w, self.fc_b, self.mlp_proj_w, self.mlp_proj_b,
                      act="gelu_tanh")
        return d, h


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config, device=torch.device("cpu"), seed: int = 1234):
        super().__init__()
        self.cfg = cfg
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        self.wte = _param((cfg.vocab_size, cfg.n_embd), 0.02, device, gen)
        self.wpe = _param((cfg.block_size, cfg.n_embd), 0.01, device, gen)
        # gradient sinks (trainer opt-in): wpe is used once per step; wte twice (input
        # embedding + tied LM head), both uses accumulate into its .grad in-kernel
        # both embedding tables get their gradient only from the embedding backward, the last
        # op of the step: the DDP trainer gives them a bucket of their own (parallel/ddp.py)
        self.wte._dlbb_late_grad = True
        self.wpe._dlbb_late_grad = True
        self._fused_embedding = os.environ.get("DLBB_EMB", "1") != "0"   # A/B switch
        if self._fused_embedding:
            self.wpe._dlbb_single_use = True
            self.wte._dlbb_sink_uses = 2
        self.blocks = nn.ModuleList([Block(cfg, device, gen) for _ in range(cfg.n_layer)])
        self.ln_f = LN(cfg.n_embd, device)

    def forward(self, idx, targets=None):
        B, T = idx.shape
        if self._fused_embedding:
            x = ops.embedding(idx, self.wte, self.wpe)
        else:
            x = torch.nn.functional.embedding(idx, self.wte) + self.wpe[:T]
        y, h = self.blocks[0].ln_1(x)
        for i, blk in enumerate(self.blocks):
            d, h = blk(y, h)
            nxt = self.blocks[i + 1].ln_1 if i + 1 < len(self.blocks) else self.ln_f
            y, h = nxt(d, residual=h)
        if targets is None:
            return linear_train(y, self.wte)
        # LM head + loss fused: one pass over the logits makes loss and dlogits together
        return ops.linear_cross_entropy(y, self.wte, targets)

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def flops_per_token(self, T: int) -> float:
        """6N + attention (12 * L * T * d) per token, the standard transformer estimate."""
        n = self.num_parameters() - self.wpe.numel()
        return 6.0 * n + 12.0 * self.cfg.n_layer * T * self.cfg.n_embd
