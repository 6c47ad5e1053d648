"""Tensor-parallel transformer (forward / inference benchmark model).

Reference ``models.py``: ``TransformerBlock`` (107-190), ``LLM`` (197-245), ``MODEL_CONFIGS``
(252-271), ``create_model`` (278-307), ``create_model_from_config`` (310-335).

Kept from the reference (workload parity): pre-LN blocks; column-parallel QKV computing all
``3H/P`` columns; the "attention" stub that keeps the first ``H/P`` columns (``models.py:162-167``)
— the GEMM reads that strided view directly (lda = 3H/P), no copy; row-parallel attention-out;
GELU (erf) MLP; 2 all-reduces per layer; final LayerNorm; ``randn`` weights (unscaled, as the
reference; ``init_std`` lets callers scale them).

MI355X-specific: all compute on-device in bf16 through the gfx950 kernels (MFMA GEMM with fused
GELU, fused residual+LayerNorm); the residual add of each sublayer is fused into the NEXT
LayerNorm, so the block is ``LN1 → QKV → out-proj → AR → (add+LN2) → up+GELU → down → AR →
(add+LN1 of the next block)``. ``attention="sdpa"`` swaps the stub for real causal attention
(torch SDPA), ``attention="flash"`` for our causal flash kernel (``ops.causal_attention``).
``overlap_chunks`` > 1 interleaves micro-batches so the all-reduces run under GEMMs (forward()).
"""

from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops import gemm as gemm_ops
from ..parallel.comm import Comm
from ..parallel.streams import concurrent_stream
from ..parallel.tensor_parallel import ColumnParallelLinear, RowParallelLinear

MODEL_CONFIGS: Dict[str, Dict[str, int]] = {
    "1B": {"hidden_size": 2048, "num_layers": 24, "num_heads": 16, "ffn_intermediate": 8192},
    "7B": {"hidden_size": 4096, "num_layers": 32, "num_heads": 32, "ffn_intermediate": 16384},
    "13B": {"hidden_size": 5120, "num_layers": 40, "num_heads": 40, "ffn_intermediate": 20480},
}


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class LayerNormParams(nn.Module):
    def __init__(self, hidden: int, device, dtype=torch.bfloat16):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden, device=device, dtype=dtype),
                                   requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(hidden, device=device, dtype=dtype),
                                 requires_grad=False)
        self.eps = 1e-5

    def forward(self, x, residual=None, kernels="hip"):
        if kernels == "torch":
            h = x + residual if residual is not None else x
            return F.layer_norm(h, (h.shape[-1],), self.weight, self.bias, self.eps), h
        y, h = ops.layernorm(x, self.weight, self.bias, self.eps, residual=residual)
        return y, (h if h is not None else x)


class TransformerBlock(nn.Module):
    def __init__(self, hidden_size: int, num_heads: int, ffn_intermediate: int, comm: Comm,
                 generator=None, init_std: float = 1.0, allreduce: str = "rccl",
                 allreduce_dtype: str = "bf16", attention: str = "slice",
                 kernels: str = "hip"):
        super().__init__()
        P = comm.world_size
        self.hidden_size, self.num_heads, self.P = hidden_size, num_heads, P
        self.attention = attention
        self.kernels = kernels
        dev = comm.device
        self.ln1 = LayerNormParams(hidden_size, dev)
        self.qkv_proj = ColumnParallelLinear(hidden_size, 3 * hidden_size, comm,
                                             generator=generator, std=init_std, kernels=kernels)
        self.out_proj = RowParallelLinear(hidden_size, hidden_size, comm, generator=generator,
                                          std=init_std, allreduce=allreduce,
                                          allreduce_dtype=allreduce_dtype, kernels=kernels)
        self.ln2 = LayerNormParams(hidden_size, dev)
        self.ffn_up = ColumnParallelLinear(hidden_size, ffn_intermediate, comm,
                                           generator=generator, std=init_std, kernels=kernels)
        self.ffn_down = RowParallelLinear(ffn_intermediate, hidden_size, comm,
                                          generator=generator, std=init_std, allreduce=allreduce,
                                          allreduce_dtype=allreduce_dtype, kernels=kernels)

    def _attn(self, qkv: torch.Tensor) -> torch.Tensor:
        hpr = self.hidden_size // self.P
        if self.attention == "slice":
            return qkv[..., :hpr]               # reference stub, models.py:166-167 (a view)
        B, S, _ = qkv.shape
        heads = self.num_heads // self.P
        hd = hpr // heads
        if self.attention == "flash" and self.kernels != "torch":
            # our causal flash kernel (csrc/attention.hip, head dim 64 / 128) straight on the
            # rank's fused [B, S, 3, heads, hd] QKV shard — no unbind / transpose copies
            return ops.causal_attention(qkv, heads)
        q, k, v = qkv.view(B, S, 3, heads, hd).permute(2, 0, 3, 1, 4).unbind(0)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return o.transpose(1, 2).reshape(B, S, hpr)

    def forward(self, y1: torch.Tensor, h: torch.Tensor):
        """``y1`` = LN1(h) (computed by the caller's fused add+LN); returns (d, h) where the
        block output is ``h + d`` (added inside the next fused LayerNorm)."""
        gen = self.steps(y1, h)
        try:
            while True:
                next(gen)
        except StopIteration as e:
            return e.value

    def steps(self, y1: torch.Tensor, h: torch.Tensor, slot: int = 0, stream=None):
        """The block as a generator that yields after launching each of its two all-reduces
        (the event to wait on before the all-reduced tensor is read; None when inline) —
        :meth:`LLM.forward` interleaves micro-batches on it. Returns ``(d, h)``."""
        qkv = self.qkv_proj(y1)
        a, ev = self.out_proj.launch(self._attn(qkv), slot, stream)
        yield ev
        y2, h = self.ln2(a, residual=h, kernels=self.kernels)          # h = h + attn_out
        u = self.ffn_up(y2, act="gelu")                                 # GELU fused (erf)
        d, ev = self.ffn_down.launch(u, slot, stream)
        yield ev
        return d, h


class LLM(nn.Module):
    def __init__(self, hidden_size: int, num_layers: int, num_heads: int, ffn_intermediate: int,
                 comm: Comm, seed: int = 0, init_std: float = 1.0, allreduce: str = "rccl",
                 allreduce_dtype: str = "bf16", attention: str = "slice", kernels: str = "hip",
                 overlap_chunks: int = 1):
        super().__init__()
        self.hidden_size, self.num_layers = hidden_size, num_layers
        # > 1: split the batch into this many micro-batches and interleave them so every
        # row-parallel all-reduce (on a side comm stream) runs under the next micro-batch's
        # GEMMs — see forward()
        self.overlap_chunks = max(1, int(overlap_chunks))
        # overlapped forward, A/B knob: each micro-batch on a compute stream of its own (so two
        # micro-batches' small per-rank GEMMs could share the chip) instead of one compute
        # stream. Measured worse (tools/diag/tp_overlap_probe.py, profiles/r03_tp): with three
        # busy streams the all-reduces stop overlapping at all (7B shard-8 at 300 GB/s: 25.0 vs
        # 18.0 ms), so the default is one compute stream + the comm stream.
        self.chunk_streams = False
        self._comm_stream = None
        self._chunk_streams = []
        self.num_heads, self.ffn_intermediate = num_heads, ffn_intermediate
        self.comm = comm
        self.world_size = comm.world_size
        self.kernels = kernels
        gen = torch.Generator(device=comm.device)
        gen.manual_seed(seed + 1000 * comm.rank)
        self.layers = nn.ModuleList([
            TransformerBlock(hidden_size, num_heads, ffn_intermediate, comm, gen, init_std,
                             allreduce, allreduce_dtype, attention, kernels)
            for _ in range(num_layers)])
        self.ln_final = LayerNormParams(hidden_size, comm.device)

    @torch.inference_mode()
    def ipc_allreduce(self):
        """The IPC all-reduce instance the row-parallel layers may use (None: RCCL only)."""
        for m in self.modules():
            car = getattr(m, "_car", None)
            if car is not None:
                return car
        return None

    def _micro_batch(self, x: torch.Tensor, slot: int = 0, stream=None):
        """One micro-batch's forward as a generator over its all-reduces (see
        :meth:`TransformerBlock.steps`); returns the final LayerNorm output."""
        if not self.layers:
            y, _ = self.ln_final(x, kernels=self.kernels)
            return y
        y, h = self.layers[0].ln1(x, kernels=self.kernels)
        for i, layer in enumerate(self.layers):
            d, h = yield from layer.steps(y, h, slot, stream)
            nxt = self.layers[i + 1].ln1 if i + 1 < len(self.layers) else self.ln_final
            y, h = nxt(d, residual=h, kernels=self.kernels)
        return y

    def overlap_split(self, x: torch.Tensor) -> int:
        """Micro-batches the forward of ``x`` runs as: ``overlap_chunks`` when the batch splits
        evenly (and the model is TP over more than one rank), else 1."""
        n = self.overlap_chunks
        if n <= 1 or self.world_size <= 1 or x.shape[0] % n:
            return 1
        return n

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """Plain: one pass, each all-reduce inline. Overlapped (``overlap_chunks`` = n > 1): the
        batch is split into n micro-batches run round-robin, each advancing to its next
        all-reduce; the all-reduce goes to a side comm stream (normal priority: a high-priority one stretches
        every compute dispatch, profiles/r03_overlap) and the micro-batch resumes only after its compute
        stream waited for it. So all-reduce k of micro-batch A runs under the GEMMs of
        micro-batch B, and every rank issues its collectives in the same order on one comm
        stream. The reference blocks on each all-reduce (models.py:95)."""
        n = self.overlap_split(x)
        if n == 1:
            gen = self._micro_batch(x)
            try:
                while True:
                    next(gen)
            except StopIteration as e:
                return e.value
        stream = None
        cur = torch.cuda.current_stream(x.device) if x.is_cuda else None
        work = [cur] * n                        # the stream each micro-batch computes on
        if x.is_cuda:
            if self._comm_stream is None:
                self._comm_stream = concurrent_stream(x.device, "tp_comm")
            stream = self._comm_stream
            # (not under HIP-graph capture: a capture forking the per-micro-batch streams crashed
            # the process on MI355X; the capture keeps one compute stream + the comm stream)
            if self.chunk_streams and not torch.cuda.is_current_stream_capturing():
                while len(self._chunk_streams) < n:
                    self._chunk_streams.append(
                        concurrent_stream(x.device, f"tp_chunk{len(self._chunk_streams)}"))
                work = self._chunk_streams[:n]
                for s in work:                  # fork: x (and last call's frees) are ready
                    s.wait_stream(cur)
        gens = [self._micro_batch(xc, slot, stream) for slot, xc in enumerate(x.chunk(n, 0))]
        pending = [None] * n
        outs = [None] * n
        live = n
        with gemm_ops.concurrent_comm():       # no persistent library GEMM beside comm kernels
            while live:
                for c in range(n):
                    if gens[c] is None:
                        continue
                    ctx = (torch.cuda.stream(work[c]) if x.is_cuda and work[c] is not cur
                           else _NullCtx())
                    with ctx:
                        if pending[c] is not None:
                            work[c].wait_event(pending[c])
                        try:
                            pending[c] = next(gens[c])
                        except StopIteration as e:
                            outs[c], gens[c], pending[c] = e.value, None, None
                            live -= 1
        if x.is_cuda:
            for s in work:                      # join
                if s is not cur:
                    cur.wait_stream(s)
        return torch.cat(outs, 0)

    @torch.no_grad()
    def load_from_dense(self, dense_state: Dict[str, torch.Tensor]) -> None:
        """Shard a world-1 model's state into this rank (Megatron layout): QKV rows are taken
        per projection (``q_r, k_r, v_r``) so the local shard is ``[q_r | k_r | v_r]`` and the
        reference's "first H/P columns" stub yields ``q_r``; FFN-up rows by block;
        row-parallel weights by column block. Used to test TP(P) == dense(1)."""
        P, r = self.world_size, self.comm.rank
        H = self.hidden_size
        for name, p in self.named_parameters():
            full = dense_state[name].to(p.device, p.dtype)
            if full.shape == p.shape:
                p.copy_(full)
            elif name.endswith("qkv_proj.weight"):
                hp = H // P
                p.copy_(torch.cat([full[j * H + r * hp: j * H + (r + 1) * hp] for j in range(3)]))
            elif name.endswith("ffn_up.weight"):
                n = p.shape[0]
                p.copy_(full[r * n:(r + 1) * n])
            elif name.endswith(("out_proj.weight", "ffn_down.weight")):
                k = p.shape[1]
                p.copy_(full[:, r * k:(r + 1) * k])
            else:
                raise KeyError(f"cannot shard {name}: {tuple(full.shape)} -> {tuple(p.shape)}")

    def get_num_parameters(self) -> int:
        """Reference formula (``models.py:240-241``): local numel × P (over-counts LN params)."""
        return sum(p.numel() for p in self.parameters()) * self.world_size

    def num_parameters_exact(self) -> int:
        local_ln = sum(p.numel() for n, p in self.named_parameters() if ".ln" in n or
                       n.startswith("ln_final"))
        local = sum(p.numel() for p in self.parameters())
        return (local - local_ln) * self.world_size + local_ln

    def get_memory_footprint(self) -> int:
        return sum(p.numel() * p.element_size() for p in self.parameters())

    def comm_bytes(self) -> int:
        return sum(m.comm_bytes for m in self.modules() if isinstance(m, RowParallelLinear))

    def flops_per_forward(self, batch: int, seq: int) -> float:
        """GEMM FLOPs of one forward on ONE rank."""
        M = batch * seq
        H, F_, P = self.hidden_size, self.ffn_intermediate, self.world_size
        per_layer = 2 * M * H * (3 * H // P) + 2 * M * (H // P) * H \
            + 2 * M * H * (F_ // P) + 2 * M * (F_ // P) * H
        return float(per_layer * self.num_layers)


def create_model(model_size: str, comm: Comm, **kw) -> LLM:
    if model_size not in MODEL_CONFIGS:
        raise ValueError(f"Invalid model size: {model_size}. Choose from {list(MODEL_CONFIGS)}")
    return LLM(comm=comm, **MODEL_CONFIGS[model_size], **kw)


def create_model_from_config(config: Dict, comm: Comm) -> LLM:
    m = config["model"]
    ex = config.get("execution", {})
    allreduce = ex.get("allreduce", "auto")
    return LLM(hidden_size=int(m["hidden_size"]), num_layers=int(m["num_layers"]),
               num_heads=int(m["num_heads"]), ffn_intermediate=int(m["ffn_intermediate"]),
               comm=comm, seed=int(config.get("input", {}).get("seed", 42)),
               init_std=float(m.get("init_std", 1.0)),
               allreduce="rccl" if allreduce in ("torch",) else allreduce,
               allreduce_dtype=ex.get("allreduce_dtype", "bf16"),
               attention=ex.get("attention", "slice"), kernels=ex.get("kernels", "hip"),
               overlap_chunks=int(ex.get("overlap_chunks", 1)))
