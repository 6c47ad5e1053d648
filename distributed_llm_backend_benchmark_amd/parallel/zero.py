"""ZeRO-2-style sharded data parallelism.

Reference: DeepSpeed ZeRO stage 2 in the smoke test ``test/ccl.py:86-96`` (gradient reduction and
optimizer-state partitioning inside ``model_engine.backward/step``), never timed there.

Built on :class:`.ddp.FlatParamTrainer`'s flat layout: every gradient bucket is padded to a
multiple of ``world x 64`` elements and split into ``world`` equal chunks; rank ``r`` owns chunk
``r`` of EVERY bucket. Per step:

* backward: each full bucket is **reduce-scattered** (RCCL ``reduce_scatter_tensor``,
  asynchronous, overlapped with the rest of backward, strictly in bucket order) into this rank's
  gradient shard;
* optimizer: ONE fused AdamW launch over the rank's fp32 master shard (1/world of the model:
  master + moments are sharded), 1/world averaging fused, writing a bf16 parameter shard;
* **all-gather** of every bucket's bf16 chunks back into the flat parameter buffer.

Traffic per step equals DDP's all-reduce (reduce-scatter + all-gather = 2(P-1)/P · bytes) while
optimizer memory drops by P.
"""

from __future__ import annotations

import contextlib

from typing import List, Tuple

import torch
import torch.distributed as dist

from ..ops import FlatAdamW
from .ddp import _ALIGN, FlatParamTrainer


class ShardedTrainer(FlatParamTrainer):
    def __init__(self, model, comm, **kw):
        if kw.get("mode", "view") != "view":
            raise ValueError("ShardedTrainer uses gradient-bucket views (mode='view')")
        if kw.get("allreduce", "rccl") != "rccl":
            raise ValueError("ShardedTrainer uses RCCL reduce-scatter / all-gather")
        super().__init__(model, comm, **kw)

    def _bucket_align(self) -> int:
        return _ALIGN * self.world

    def _init_optimizer(self, lr, betas, weight_decay) -> None:
        P = self.world
        r = self.comm.rank if self.comm is not None else 0
        self._chunks: List[Tuple[int, int, int]] = []   # (bucket src offset, shard offset, n)
        off = 0
        for b in self.buckets:
            n = (b.end - b.start) // P
            self._chunks.append((b.start + r * n, off, n))
            off += n
        self.shard_numel = off
        dev = self.flat_param.device
        master = torch.empty(off, dtype=torch.float32, device=dev)
        for src, dst, n in self._chunks:
            master[dst:dst + n].copy_(self.flat_param[src:src + n].float())
        self.master = master
        self.grad_shard = torch.zeros(off, dtype=self.flat_grad.dtype, device=dev)
        self.param_shard = torch.empty(off, dtype=torch.bfloat16, device=dev)
        self.opt = FlatAdamW(master, lr=lr, betas=betas, weight_decay=weight_decay)

    def _launch(self, b) -> None:
        b.launched = True
        src, dst, n = self._chunks[b.idx]
        out = self.grad_shard[dst:dst + n]
        ws = self._wgrad_stream
        if ws is not None:
            # bucket complete on main AND side stream (sink weight gradients): issue from the
            # side stream after it joined the main one; finish() joins it back
            ws.wait_stream(torch.cuda.current_stream(out.device))
            for other in self._wgrad_streams[1:]:
                ws.wait_stream(other)
        with torch.cuda.stream(ws) if ws is not None else contextlib.nullcontext():
            if self.world == 1:
                out.copy_(self.flat_grad[b.start:b.end])
                return
            b.work = dist.reduce_scatter_tensor(out, self.flat_grad[b.start:b.end],
                                                async_op=True)

    def _optimizer_step(self) -> None:
        self.opt.step(self.grad_shard, working_bf16=self.param_shard,
                      grad_scale=1.0 / self.world)
        self._gather_params()

    def _replicated_state(self) -> bool:
        return False

    def _refresh_params(self) -> None:
        self.param_shard.copy_(self.master.to(torch.bfloat16))
        self._gather_params()

    def _gather_params(self) -> None:
        works = []
        for b, (src, dst, n) in zip(self.buckets, self._chunks):
            shard = self.param_shard[dst:dst + n]
            full = self.flat_param[b.start:b.end]
            if self.world == 1:
                full.copy_(shard)
            else:
                works.append(dist.all_gather_into_tensor(full, shard, async_op=True))
        for w in works:
            w.wait()
