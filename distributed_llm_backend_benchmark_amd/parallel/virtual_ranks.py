"""Single-process N-virtual-rank harness for the IPC xGMI collectives.

``gpurun`` gives one MI355X per call, so the one-shot / two-shot / registered / push all-reduce
and the direct all-gather / reduce-scatter / all-to-all kernels of ``csrc/custom_allreduce.hip``
cannot run across GPUs here. This harness runs them on ONE GPU with W virtual ranks: W
``CarState`` objects created in this process (``dlbb_car_create(r, W, cap)``), each opened with
its siblings' own allocations as "peer" buffers (``dlbb_car_open_local`` — no IPC handles).

Two launch forms, both executing the production device code:

* ``fused`` (default): ONE launch of ``W x nblocks`` workgroups; workgroup ``g`` plays rank
  ``g // nblocks`` (``dlbb_car_vr_launch``). All ranks are co-resident by construction — the
  launcher refuses grids larger than the device's resident capacity for that kernel.
* ``streams``: the per-rank production launch (``dlbb_car_allreduce`` etc.) of every rank on its
  own HIP stream, i.e. W concurrent kernels exactly as W processes would enqueue them. Needs
  ``W <= GPU_MAX_HW_QUEUES`` (4 here) distinct hardware queues, so the W streams are picked by
  a concurrency probe (``parallel.streams.concurrent_group``): two ranks on one queue serialize,
  the first waits out its wall-clock bound (``custom_allreduce.set_timeout_ms``) and flags the
  timeout, which :meth:`errors` reports — never a hang.

What the numbers mean: every byte a real rank would move over xGMI moves through the one
GPU's HBM here, so the harness measures the kernels' protocol cost (flag round trip, epoch and
barrier overhead: the small-message latency floor) and their memory-level parallelism (large
messages, against the HBM roofline), not xGMI link bandwidth.
"""

from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import torch

from ..ops import _lib
from .streams import concurrent_group

K_ONESHOT, K_TWOSHOT, K_REG, K_PUSH, K_AG, K_A2A, K_RS = 1, 2, 3, 4, 5, 6, 7
KIND_NAMES = {K_ONESHOT: "oneshot", K_TWOSHOT: "twoshot", K_REG: "reg_pull", K_PUSH: "reg_push",
              K_AG: "allgather", K_A2A: "alltoall", K_RS: "reduce_scatter"}
HIP_ERROR_INVALID_CONFIGURATION = 9


def _ptrs(ts: Sequence[Optional[torch.Tensor]]):
    arr = (ctypes.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = None if t is None else t.data_ptr()
    return arr


class VirtualRanks:
    """W virtual ranks of the custom collectives on the current HIP device."""

    def __init__(self, world: int, capacity_bytes: int = 64 << 20,
                 device: Optional[torch.device] = None):
        if not 2 <= world <= 8:
            raise ValueError("virtual ranks: 2 <= world <= 8")
        self.lib = _lib.lib()
        self.world = world
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.states: List[ctypes.c_void_p] = []
        try:
            with torch.cuda.device(self.device):
                for r in range(world):
                    h = ctypes.c_void_p()
                    _lib.check(self.lib.dlbb_car_create(r, world, int(capacity_bytes),
                                                        ctypes.byref(h)), "car_create")
                    self.states.append(h)
                self._arr = (ctypes.c_void_p * world)(*[h.value for h in self.states])
                _lib.check(self.lib.dlbb_car_open_local(self._arr, world), "car_open_local")
        except BaseException:
            self.close()
            raise
        self.capacity = int(self.lib.dlbb_car_capacity(self.states[0]))
        self._keep: List[torch.Tensor] = []

    # ------------------------------------------------------------------ capacity
    def max_blocks(self, kind: int, dtype: torch.dtype = torch.bfloat16) -> int:
        """Largest per-rank workgroup count the fused launch accepts for ``kind``."""
        with torch.cuda.device(self.device):
            cap = int(self.lib.dlbb_car_vr_max_blocks(kind, _lib.dt(torch.empty(0, dtype=dtype)),
                                                      self.world))
        return min(256, cap // self.world)

    # ------------------------------------------------------------------ fused launches
    def launch(self, kind: int, count: int, dtype: torch.dtype, nblocks: int,
               inputs: Optional[Sequence[torch.Tensor]] = None,
               outputs: Optional[Sequence[torch.Tensor]] = None, reg_id: int = -1,
               stream: Optional[torch.cuda.Stream] = None) -> None:
        """One fused launch of collective ``kind`` for all W ranks. ``count``: elements for
        the all-reduce kinds, bytes for the direct kinds (the C entry points' units)."""
        st = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        ins = _ptrs(inputs) if inputs is not None else None
        outs = _ptrs(outputs) if outputs is not None else None
        rc = self.lib.dlbb_car_vr_launch(self._arr, self.world, kind, ins, outs, int(count),
                                         _lib.dt(torch.empty(0, dtype=dtype)), int(reg_id),
                                         int(nblocks), st)
        if rc == HIP_ERROR_INVALID_CONFIGURATION:
            raise ValueError(f"{self.world} x {nblocks} workgroups of {KIND_NAMES[kind]} exceed "
                             f"the resident capacity (max {self.max_blocks(kind, dtype)} per rank)")
        _lib.check(rc, f"car_vr_launch({KIND_NAMES[kind]})")

    def all_reduce(self, inputs: Sequence[torch.Tensor], outputs: Sequence[torch.Tensor],
                   algo: int = K_ONESHOT, nblocks: int = 32) -> None:
        self._check_list(inputs)
        self._check_list(outputs)
        self.launch(algo, inputs[0].numel(), inputs[0].dtype, nblocks, inputs, outputs)

    def register(self, bufs: Sequence[torch.Tensor]) -> int:
        """Register one buffer per virtual rank (same numel / dtype) under one id."""
        self._check_list(bufs)
        rid = ctypes.c_int(-1)
        nbytes = bufs[0].numel() * bufs[0].element_size()
        _lib.check(self.lib.dlbb_car_reg_local(self._arr, self.world, _ptrs(bufs), nbytes,
                                               ctypes.byref(rid)), "car_reg_local")
        self._keep.extend(bufs)
        return int(rid.value)

    def all_reduce_registered(self, bufs: Sequence[torch.Tensor], rid: int, nblocks: int = 64,
                              push: bool = False) -> None:
        self.launch(K_PUSH if push else K_REG, bufs[0].numel(), bufs[0].dtype, nblocks,
                    reg_id=rid)

    def direct(self, kind: int, bufs: Sequence[torch.Tensor], rid: int,
               outputs: Sequence[torch.Tensor], nblocks: int = 64) -> None:
        """all-gather (chunk = whole input), all-to-all (chunk = input / W) or reduce-scatter
        (input split W ways) from the registered ``bufs`` into ``outputs``."""
        b = bufs[0].numel() * bufs[0].element_size()
        count = b // self.world if kind == K_A2A else b
        self.launch(kind, count, bufs[0].dtype, nblocks, outputs=outputs, reg_id=rid)

    # ------------------------------------------------------------------ per-rank streams
    def all_reduce_streams(self, inputs: Sequence[torch.Tensor], outputs: Sequence[torch.Tensor],
                           streams: Sequence[torch.cuda.Stream], algo: int = K_ONESHOT,
                           nblocks: int = 32) -> None:
        """The production per-rank launch of every rank on its own stream (see module doc)."""
        self._check_list(inputs)
        for r in range(self.world):
            _lib.check(self.lib.dlbb_car_allreduce(
                self.states[r], inputs[r].data_ptr(), outputs[r].data_ptr(), inputs[r].numel(),
                _lib.dt(inputs[r]), algo, nblocks, streams[r].cuda_stream), "car_allreduce")

    # ------------------------------------------------------------------ health
    def errors(self) -> List[int]:
        """Per-rank timeout flags (read and cleared; synchronous)."""
        return [int(self.lib.dlbb_car_error(h)) for h in self.states]

    def _check_list(self, ts: Sequence[torch.Tensor]) -> None:
        if len(ts) != self.world:
            raise ValueError(f"need one tensor per virtual rank ({self.world}), got {len(ts)}")
        n, dt = ts[0].numel(), ts[0].dtype
        for t in ts:
            if t.numel() != n or t.dtype != dt or not t.is_contiguous() or t.device != self.device:
                raise ValueError("virtual-rank tensors must share numel, dtype and device and "
                                 "be contiguous")

    def close(self) -> None:
        for h in getattr(self, "states", []):
            if h:
                self.lib.dlbb_car_destroy(h)
        self.states = []
        self._keep = []

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def time_calls(fn, iters: int, stream: Optional[torch.cuda.Stream] = None) -> float:
    """Mean microseconds per call of ``iters`` back-to-back calls between two events."""
    st = stream or torch.cuda.current_stream()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(iters):
        fn()
    e.record(st)
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def time_streams(V: "VirtualRanks", xs, outs, streams, algo: int, nblocks: int,
                 iters: int) -> float:
    """Mean microseconds per call of the per-rank production launch (every rank's kernel on its
    own stream, back to back), event-timed: all streams start behind one event and the clock
    stops when the last stream drains."""
    cur = torch.cuda.current_stream()
    for _ in range(3):
        V.all_reduce_streams(xs, outs, streams, algo=algo, nblocks=nblocks)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(cur)
    for st in streams:
        st.wait_event(s)
    for _ in range(iters):
        V.all_reduce_streams(xs, outs, streams, algo=algo, nblocks=nblocks)
    for st in streams:
        ev = torch.cuda.Event()
        ev.record(st)
        cur.wait_event(ev)
    e.record(cur)
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def emulation_summary(worlds=(2, 4, 8), small_bytes: int = 512,
                      big_bytes: int = 64 << 20) -> dict:
    """Validated single-GPU emulation numbers for bench.py's world-1 line: one-shot all-reduce
    latency at ``small_bytes`` and the registered in-place two-shot at ``big_bytes`` (the headline
    message) for W virtual ranks. Every configuration is first checked against an fp32 sum of the
    rank inputs; a failing one is reported as invalid, never timed.

    The one-shot latency comes in two forms: ``oneshot_<n>B`` is ONE fused grid for all W ranks
    (protocol floor), ``oneshot_<n>B_per_rank_launch`` the production path — each rank's own
    launch on its own stream, as W processes enqueue it (W <= 4 hardware queues on this box)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    out = {}
    for W in worlds:
        V = VirtualRanks(W, capacity_bytes=max(small_bytes, 1 << 20))
        try:
            rec = {}
            for kind, nbytes, nb, iters in ((K_ONESHOT, small_bytes, 1, 200),
                                            (K_REG, big_bytes, None, 10)):
                xs = []
                for r in range(W):
                    g = torch.Generator(device=dev)
                    g.manual_seed(1000 * W + r)
                    xs.append(torch.randn(nbytes // 2, generator=g, device=dev)
                              .to(torch.bfloat16))
                ref = sum(x.float() for x in xs)
                nb = nb or V.max_blocks(kind)
                if kind == K_REG:
                    bufs = [x.clone() for x in xs]
                    rid = V.register(bufs)
                    V.all_reduce_registered(bufs, rid, nblocks=nb)
                    got = bufs
                else:
                    got = [torch.empty_like(x) for x in xs]
                    V.all_reduce(xs, got, algo=kind, nblocks=nb)
                torch.cuda.synchronize()
                ok = not any(V.errors()) and all(
                    torch.allclose(g_.float(), ref, rtol=2e-2, atol=5e-2 * W) for g_ in got)
                key = f"{KIND_NAMES[kind]}_{nbytes}B"
                if not ok:
                    rec[key] = {"valid": False}
                    continue
                if kind == K_REG:
                    for b in bufs:
                        b.zero_()
                    # CU budget per rank: best of a few (all within the resident capacity)
                    cands = sorted({min(32, nb), min(64, nb), nb})
                    times = {c: time_calls(lambda c=c: V.all_reduce_registered(
                        bufs, rid, nblocks=c), iters) for c in cands}
                    nb = min(times, key=times.get)
                    us = times[nb]
                else:
                    us = time_calls(lambda: V.all_reduce(xs, got, algo=kind, nblocks=nb), iters)
                rec[key] = {"valid": not any(V.errors()), "us": round(us, 2), "nblocks": nb}
                if kind == K_ONESHOT and W <= 4:
                    # W streams on W distinct hardware queues (parallel/streams.py): two
                    # ranks on one queue would serialise behind each other's spin-waits
                    sts = concurrent_group(torch.device("cuda", torch.cuda.current_device()),
                                           W, "virtual_ranks")
                    for g_ in got:
                        g_.zero_()
                    V.all_reduce_streams(xs, got, sts, algo=kind, nblocks=nb)
                    torch.cuda.synchronize()
                    ok = not any(V.errors()) and all(
                        torch.allclose(g_.float(), ref, rtol=2e-2, atol=5e-2 * W) for g_ in got)
                    pk = f"{key}_per_rank_launch"
                    if ok:
                        us_s = time_streams(V, xs, got, sts, kind, nb, iters)
                        rec[pk] = {"valid": not any(V.errors()), "us": round(us_s, 2),
                                   "nblocks": nb, "streams": W}
                    else:
                        rec[pk] = {"valid": False}
                del xs, got, ref
            out[f"W{W}"] = rec
        finally:
            V.close()
    return out
