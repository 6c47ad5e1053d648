"""Megatron-1D tensor-parallel linears.

Reference: ``ColumnParallelLinear`` (``models.py:19-47``; out-features sharded, ``:33``) and
``RowParallelLinear`` (``models.py:50-100``; in-features sharded, ``:66``; partial outputs
summed by ``comm.Allreduce`` on fp32 host numpy buffers, ``:84-98``).

MI355X design:
* weights are stored ``[out, in]`` (K-contiguous, MFMA-native) bf16 on the device;
* the GEMM is the hand-written MFMA kernel (``ops.linear``) with GELU fused into the
  column-parallel FFN-up epilogue;
* the row-parallel partial sum is all-reduced ON DEVICE: bf16 over RCCL by default, or the
  reference's fp32 wire format (GEMM epilogue writes fp32 directly — no cast pass), or the IPC
  one-shot/two-shot xGMI kernel; the residual add is NOT done here but fused into the next
  LayerNorm (``ops.layernorm(x, residual=...)``).
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import ops
from .comm import Comm


def _randn_weight(out_f: int, in_f: int, device, dtype, generator, std: float) -> nn.Parameter:
    w = torch.empty(out_f, in_f, device=device, dtype=torch.float32)
    w.normal_(0.0, std, generator=generator)
    return nn.Parameter(w.to(dtype), requires_grad=False)


class ColumnParallelLinear(nn.Module):
    """y_local = act(x @ W_local^T); W_local = rows [rank*out/P, (rank+1)*out/P) of W."""

    def __init__(self, in_features: int, out_features: int, comm: Comm,
                 dtype=torch.bfloat16, generator=None, std: float = 1.0,
                 kernels: str = "hip"):
        super().__init__()
        P = comm.world_size
        if out_features % P:
            raise ValueError(f"out_features {out_features} not divisible by world {P}")
        self.in_features, self.out_features = in_features, out_features
        self.out_per_rank = out_features // P
        self.kernels = kernels
        self.weight = _randn_weight(self.out_per_rank, in_features, comm.device, dtype,
                                    generator, std)

    def forward(self, x: torch.Tensor, act: Optional[str] = None) -> torch.Tensor:
        if self.kernels == "torch":
            y = x @ self.weight.t()
            return torch.nn.functional.gelu(y) if act else y
        return ops.linear(x, self.weight, act=act)


class RowParallelLinear(nn.Module):
    """y = allreduce_sum(x_local @ W_local^T); W_local = columns of W for this rank's shard."""

    def __init__(self, in_features: int, out_features: int, comm: Comm,
                 dtype=torch.bfloat16, generator=None, std: float = 1.0,
                 allreduce: str = "rccl", allreduce_dtype: str = "bf16",
                 kernels: str = "hip"):
        super().__init__()
        P = comm.world_size
        if in_features % P:
            raise ValueError(f"in_features {in_features} not divisible by world {P}")
        self.comm = comm
        self.in_features, self.out_features = in_features, out_features
        self.in_per_rank = in_features // P
        self.allreduce = allreduce
        self.allreduce_dtype = allreduce_dtype
        self.kernels = kernels
        self.weight = _randn_weight(out_features, self.in_per_rank, comm.device, dtype,
                                    generator, std)
        self._car = None
        self._native = None
        if allreduce in ("custom", "auto") and comm.is_gpu and comm.world_size > 1:
            from .custom_allreduce import get_custom_allreduce

            self._car = get_custom_allreduce(comm)
        if allreduce in ("native", "auto") and comm.is_gpu and comm.world_size > 1:
            # RCCL enqueued on the compute stream by our engine: no ProcessGroupNCCL stream hop
            # and HIP-graph capturable (run_tp --graph at world > 1)
            from .rccl_native import get_native

            try:
                self._native = get_native(comm)
            except RuntimeError:
                if allreduce == "native":
                    raise
        self.comm_bytes = 0   # bytes all-reduced by this layer (accounting)
        # allreduce="emulate" (run_tp --shard-as P: ONE GPU runs rank 0's shard of a P-way
        # model): the partial sum goes through a stand-in with the local HBM traffic of one
        # rank's one-shot all-reduce (P inputs read, 1 written: y + (P-1) zero buffers) and,
        # with `emulate_busbw` GB/s, then holds `emulate_blocks` workgroups for the ring time
        # bytes * 2(P-1)/P / busBW — the link-bound duration (parallel/ddp.py uses the same model)
        self.emulate_busbw: Optional[float] = None
        self.emulate_blocks = 32
        self._emu_zeros: Optional[torch.Tensor] = None
        self._events = {}     # micro-batch slot -> (ready, done) events (overlapped forward)

    def _emulated_all_reduce(self, t: torch.Tensor) -> None:
        from ..ops.elementwise import reduce_sum, spin_ns

        P = self.comm.world_size
        n = t.numel()
        if self._emu_zeros is None or self._emu_zeros.numel() < n \
                or self._emu_zeros.dtype != t.dtype:
            self._emu_zeros = torch.zeros(n, dtype=t.dtype, device=t.device)
        flat = t.view(-1)
        reduce_sum([flat] + [self._emu_zeros[:n]] * (P - 1), out=flat)
        if self.emulate_busbw:
            nbytes = n * t.element_size()
            spin_ns(int(nbytes * 2.0 * (P - 1) / P / self.emulate_busbw), self.emulate_blocks,
                    t.device)

    # ---- registered output buffer: the GEMM writes the partial sum straight into a buffer every
    # rank IPC-mapped once, and the in-place registered two-shot reduces it there — no copy into
    # the staging buffer, no capacity limit. The IPC instance owns one buffer per (shape, dtype),
    # shared by every row-parallel layer of the model: the forward is sequential on one stream and
    # each output is consumed (next LayerNorm) before the next row-parallel GEMM rewrites it, and
    # the kernel's exit barrier (phase 2) guarantees no peer still reads it by then.
    def _registered_out(self, shape, dtype, slot: int = 0) -> Optional[tuple]:
        car = self._car
        if car is None or not car.reg_healthy or self.allreduce not in ("custom", "auto"):
            return None
        numel = 1
        for d in shape:
            numel *= int(d)
        esz = torch.tensor([], dtype=dtype).element_size()
        nbytes = numel * esz
        if nbytes <= car.oneshot_max:          # small (decode): staged one-shot is faster
            return None
        if nbytes % (8 * esz * self.comm.world_size):
            return None
        limit = getattr(car, "reg_max", None)  # calibrated: registered beats RCCL up to here
        if self.allreduce == "auto" and nbytes > (limit if limit is not None else car.auto_max):
            return None
        return car.registered_buffer(numel, dtype, slot)   # collective on first use

    def _all_reduce(self, t: torch.Tensor) -> None:
        self.comm_bytes += t.numel() * t.element_size()
        if self.comm.world_size == 1:
            return
        if self.allreduce == "emulate":
            self._emulated_all_reduce(t)
            return
        car = self._car
        if car is not None and (self.allreduce == "custom" or car.should_use(t)) \
                and car.supports(t):
            car.all_reduce_(t)
        elif self._native is not None and t.is_contiguous():
            self._native.enqueue("allreduce", t, t, t.numel())
        else:
            dist.all_reduce(t)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """Public API: always an OWNED tensor. (The zero-copy :meth:`launch` may return a view
        of the IPC-registered output buffer, which every same-shape row-parallel layer shares and
        the next call rewrites — ADVICE r03; only the model's block, which consumes each output
        in the next LayerNorm, uses that path.)"""
        y, _ = self.launch(x)
        if self._aliases_registered(y):
            y = y.clone()
        return y

    def _aliases_registered(self, y: torch.Tensor) -> bool:
        car = self._car
        if car is None or not y.is_cuda:
            return False
        p = y.data_ptr()
        for buf, _ in car._owned.values():
            base = buf.data_ptr()
            if base <= p < base + buf.numel() * buf.element_size():
                return True
        return False

    def launch(self, x: torch.Tensor, slot: int = 0, stream=None):
        """Internal zero-copy path (TransformerBlock): GEMM on the current stream, then the
        all-reduce — on ``stream`` when given (a
        side comm stream: returns ``(y, event)``, and the caller makes its stream wait on the
        event before reading ``y``; the overlapped TP forward runs another micro-batch's GEMMs
        meanwhile), else inline (``event`` None). ``slot``: which registered output buffer (one
        per micro-batch in flight). With a registered output, ``y`` is a view of a buffer shared
        by every same-shape row-parallel layer: consume it before the next row-parallel call."""
        fp32_wire = self.allreduce_dtype == "fp32"
        if self.kernels == "torch":
            y = x @ self.weight.t()
            if fp32_wire:
                y = y.float()
            return self._reduce_then(y, x.dtype, None, stream, slot)
        odt = torch.float32 if fp32_wire else x.dtype
        reg = (self._registered_out((*x.shape[:-1], self.out_features), odt, slot)
               if self.comm.world_size > 1 and x.is_cuda else None)
        if reg is not None:
            buf, rid = reg
            y = buf.view(*x.shape[:-1], self.out_features)
            ops.linear(x, self.weight, out_dtype=odt, out=y)
        else:
            y = ops.linear(x, self.weight, out_dtype=odt)
        return self._reduce_then(y, x.dtype, reg, stream, slot)

    def _reduce_then(self, y, out_dtype, reg, stream, slot=0):
        def reduce_and_cast():
            if reg is not None:
                self.comm_bytes += y.numel() * y.element_size()
                self._car.all_reduce_registered(reg[0], reg[1])
            else:
                self._all_reduce(y)
            if y.dtype == out_dtype:
                return y
            if self.kernels == "torch":
                return y.to(out_dtype)
            return ops.cast(y, out_dtype)   # HIP cast kernel (reference models.py:98)

        if stream is None or not y.is_cuda:
            return reduce_and_cast(), None
        # two events per micro-batch slot, reused every call (host cost: the overlapped forward
        # issues 2 x layers x micro-batches of these): each is waited on before it is recorded
        # again — `ready` by the comm stream right below, `done` by the caller before it
        # resumes this micro-batch
        evs = self._events.get(slot)
        if evs is None:
            evs = self._events[slot] = (torch.cuda.Event(), torch.cuda.Event())
        ready, done = evs
        ready.record(torch.cuda.current_stream(y.device))
        stream.wait_event(ready)                # the partial sum is complete
        with torch.cuda.stream(stream):
            out = reduce_and_cast()
            done.record(stream)
        return out, done
