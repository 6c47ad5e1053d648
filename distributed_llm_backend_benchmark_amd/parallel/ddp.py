"""Data-parallel training with bucketed gradient all-reduce overlapped with backward.

The reference's data parallelism is DeepSpeed's engine in smoke tests only
(``test/ccl.py:74-115`` ZeRO-2, ``test/ds_mpi_test.py:13-47``, ``test/test.py:16-41``); the
gradient reduction happens inside ``model_engine.backward`` and is never timed. This module is
the MI355X-native replacement used by the GPT-2 DDP microbenchmark:

* **Flat buffers, sized for 288 GB HBM.** All trainable parameters live in ONE flat bf16 buffer
  (params become views), with ONE fp32 master copy and ONE flat bf16 gradient buffer whose
  slices are the parameters' ``.grad`` — autograd accumulates straight into the buckets, so no
  flatten/copy pass exists at all (``mode="view"``). ``mode="flatten"`` instead lets autograd
  allocate grads and copies each ready bucket with the one-launch multi-tensor chunk-copy kernel.
* **Buckets in backward order** (parameters laid out in reverse registration order), capped at
  ``bucket_mb`` (default 64 MiB: on xGMI the ring all-reduce is link-bound, so few large
  buckets amortise RCCL launch/protocol cost; still several buckets so the first all-reduce
  starts early in backward).
* **Overlap**: a post-accumulate-grad hook counts ready params; a full bucket is all-reduced
  asynchronously (RCCL runs on ProcessGroupNCCL's own stream, ordered after the
  producing kernels by an event), strictly in bucket order on every rank (identical collective
  order — RCCL would hang otherwise). ``finish()`` waits the works; the optimizer consumes the
  reduced flat gradient with the 1/world average fused into the AdamW kernel.
* ``allreduce="custom"`` routes buckets through the IPC xGMI kernel (in place on the
  IPC-registered bucket when the registered self-test passed, else via its staging buffer), and
  ``allreduce="native"`` through our own RCCL communicator (``rccl_native``), both on a
  dedicated comm stream instead of ProcessGroupNCCL's. That stream has NORMAL priority: at high
  priority its workgroups took CU slots ahead of the backward's hipBLASLt Stream-K GEMMs, whose
  persistent grids then stalled (+69 % step time in 4 of 15 settings;
  profiles/r02_overlap/SUMMARY.md). ``comm_blocks`` is the reductions' CU budget.
"""

from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import FlatAdamW
from ..ops.elementwise import ChunkTable, ScaleTable, reduce_sum, spin_ns
from ..ops.xent import mark_unit_upstream
from ..utils import tracing
from .comm import Comm
from .streams import concurrent_stream, fork, runs_concurrently

# sink dW GEMMs on a side stream (default on; DLBB_WGRAD_STREAM=0 for the A/B). Rounds 1-2
# measured +4 % step time on GPT-2 with a pool stream; since the side streams are chosen by the
# concurrency probe (parallel/streams.py: a pool stream could share the compute stream's
# hardware queue) the weight gradients fill the CUs the 192-tile dgrad grids leave idle: 19.30 ->
# 18.90 ms, and 19.17 -> 18.58 ms with the interleaved autotune timing
# (profiles/r03_lean/tune_ab). Not adopted and removed in round 6: several
# weight-gradient streams, CU-masked side streams (2.7-3x slower), side / comm stream
# priorities (high-priority comm stretched every dispatch, profiles/r03_overlap), the early
# AdamW of untouched embedding rows (no gain, profiles/r05_step §11).
_WGRAD_STREAM = os.environ.get("DLBB_WGRAD_STREAM", "1") == "1"
# split optimizer only: AdamW of a head bucket is issued as soon as that bucket is reduced,
# during backward, on a stream of its own (1) or on the weight-gradient side stream (2, default),
# instead of for all head buckets after backward (0). GPT-2 step, three interleaved reps in one
# call: 0 -> 17.45-17.47 ms, 1 -> 17.48-17.52, 2 -> 17.42-17.43 (profiles/r05_step/SUMMARY.md §5):
# the AdamW ranges slot in behind the side stream's weight gradients instead of competing with
# the main stream from a fourth queue. Bit-exact in every mode (tests/test_comm_gpu.py).
# World > 1 keeps 0 unless set: there mode 2 would hold every later weight gradient behind the
# bucket's all-reduce (the AdamW range waits for it on that stream), and mode 1 is unmeasured
# across GPUs.
_OPT_OVERLAP = os.environ.get("DLBB_OPT_OVERLAP")
_ALIGN = 64  # elements: keeps every param view 128-B aligned (16-B MFMA/glds rows)


class _Bucket:
    def __init__(self, idx: int, start: int, end: int, params: List[torch.nn.Parameter]):
        self.idx, self.start, self.end = idx, start, end
        self.params = params
        self.ready = 0
        self.launched = False
        self.work = None
        self.done_event = None
        self.table: Optional[ChunkTable] = None
        self.table_key = None
        self.opt_done = False       # its AdamW range already queued this step


class FlatParamTrainer:
    def __init__(self, model: torch.nn.Module, comm: Optional[Comm], lr: float = 3e-4,
                 betas=(0.9, 0.95), weight_decay: float = 0.0, bucket_mb: float = 64.0,
                 overlap: bool = True, mode: str = "view", allreduce: str = "rccl",
                 grad_dtype: torch.dtype = torch.bfloat16, comm_blocks: Optional[int] = None,
                 emulate_comm=False, emulate_world: int = 8, split_optimizer: bool = True,
                 late_bucket: bool = True):
        if mode == "view" and grad_dtype != torch.bfloat16:
            raise ValueError("grad_dtype must be the parameter dtype (bf16) in mode='view': "
                             "autograd accumulates straight into the bucket views; use "
                             "mode='flatten' for fp32 gradient buckets")
        self.model = model
        self.comm = comm
        self.world = comm.world_size if comm is not None else 1
        self.overlap = overlap
        self.mode = mode
        self.allreduce = allreduce
        params = []
        seen = set()
        for p in model.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        order = list(reversed(params))          # backward produces grads roughly in reverse
        dev = params[0].device
        # layout: params back to back (each 64-element aligned), buckets closed at >= cap and
        # padded to a multiple of `bucket_align` elements (ZeRO shards need P-divisible buckets)
        cap = int(bucket_mb * (1 << 20) / torch.tensor([], dtype=grad_dtype).element_size())
        balign = max(_ALIGN, self._bucket_align())
        # Params whose gradient completes only at the very END of backward (model opt-in
        # ``_dlbb_late_grad``: the embedding tables — the embedding backward is the step's last
        # op) start a bucket of their own, so the bucket all-reduced after backward holds only
        # them, not the last blocks' gradients too (GPT-2's tail bucket was
        # blocks 1-0 + the tied 77 MB wte, ~43 % of the gradient bytes).
        offs, spans, cur, start, total = [], [], [], 0, 0
        def is_late(q):
            return late_bucket and getattr(q, "_dlbb_late_grad", False)

        for i, p in enumerate(order):
            if is_late(p) and cur and not any(is_late(q) for q in cur):
                total = (total + balign - 1) // balign * balign
                spans.append((start, total, cur))
                cur, start = [], total
            offs.append(total)
            total += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
            cur.append(p)
            if total - start >= cap or i == len(order) - 1:
                total = (total + balign - 1) // balign * balign
                spans.append((start, total, cur))
                cur, start = [], total
        self.numel = total
        self.flat_param = torch.zeros(total, dtype=torch.bfloat16, device=dev)
        self.flat_grad = torch.zeros(total, dtype=grad_dtype, device=dev)
        with torch.no_grad():
            for p, o in zip(order, offs):
                view = self.flat_param[o:o + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
        self.buckets: List[_Bucket] = []
        self._bucket_of = {}
        for st, en, ps in spans:
            self._add_bucket(st, en, ps)
        self._init_optimizer(lr, betas, weight_decay)
        self._offsets = {id(p): o for p, o in zip(order, offs)}
        self._params = order
        # weight-gradient GEMMs of sink params run on this side stream (off the backward's
        # critical path); bucket reductions and the optimizer are ordered after it
        side_ok = mode == "view" and dev.type == "cuda" and _WGRAD_STREAM
        self._wgrad_stream = concurrent_stream(dev, "ddp_wgrad") if side_ok else None
        self._wgrad_streams = [self._wgrad_stream] if self._wgrad_stream is not None else []
        n_sink = 0
        if mode == "view":
            for p, o in zip(order, offs):
                p.grad = self.flat_grad[o:o + p.numel()].view_as(p)
                # single-use params (model opt-in): backward accumulates into the bucket view
                # in-kernel and reports readiness itself (ops.linear_fn gradient sinks)
                # (a param used n > 1 times per step opts in with _dlbb_sink_uses = n, e.g. a
                # tied embedding / LM head: ready after its last use, ops.linear_fn.sink_used)
                if (getattr(p, "_dlbb_single_use", False)
                        or getattr(p, "_dlbb_sink_uses", 0) > 0):
                    p._dlbb_grad_sink = self._on_grad
                    if self._wgrad_stream is not None:
                        p._dlbb_grad_stream = self._wgrad_streams[n_sink % len(
                            self._wgrad_streams)]
                        n_sink += 1
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in order]
        self._next = 0
        self._seen = set()
        self._comm_stream = None
        self._car = None
        self._native = None
        self._bucket_reg: Dict[int, int] = {}
        if allreduce == "custom" and comm is not None and comm.is_gpu and self.world > 1:
            from .custom_allreduce import get_custom_allreduce

            self._car = get_custom_allreduce(comm)
            self._comm_stream = concurrent_stream(dev, "ddp_comm", 0)
            # buckets are fixed slices of flat_grad: IPC-map them once, then every bucket
            # all-reduce is the in-place two-shot (no staging copy, no capacity limit)
            if self._car is not None and self._car.reg_healthy:
                for b in self.buckets:
                    buf = self.flat_grad[b.start:b.end]
                    if self._car.supports_registered(buf):
                        self._bucket_reg[b.idx] = self._car.register(buf)
        if allreduce == "native" and comm is not None and comm.is_gpu and self.world > 1:
            from .rccl_native import get_native

            self._native = get_native(comm)
            self._comm_stream = concurrent_stream(dev, "ddp_comm", 0)
        if allreduce == "auto" and comm is not None and comm.is_gpu and self.world > 1:
            self._setup_auto(comm, dev)
        # CU budget of the bucket reductions that run beside backward: workgroups per IPC /
        # emulated reduction launch (None = the kernel's own size heuristic)
        self.comm_blocks = comm_blocks
        # world 1 only: every ready bucket runs a stand-in reduction on the comm
        # stream — the local HBM traffic of one rank's all-reduce (read 2n, write n: bucket +
        # zeros -> bucket, so gradients are unchanged) — to measure what overlapped bucket
        # reductions cost the backward pass on one GPU (tools/ddp_overlap.py)
        # emulate_comm=<GB/s> (a float) additionally makes each stand-in LINK-BOUND: after the
        # local traffic, `comm_blocks` (default 32) workgroups hold their CU slots for the time a
        # ring all-reduce of the bucket takes at that bus bandwidth over `emulate_world` ranks,
        # bytes * 2(P-1)/P / busBW — so an exposed tail and long-resident comm workgroups show
        # up on one GPU.
        self._emu_zero = None
        self._emu_gbps = None
        self._emu_world = int(emulate_world)
        if emulate_comm:
            if self.world != 1 or dev.type != "cuda":
                raise ValueError("emulate_comm is a single-GPU measurement (world 1, HIP device)")
            self._comm_stream = concurrent_stream(dev, "ddp_comm", 0)
            self._emu_zero = torch.zeros(max(b.end - b.start for b in self.buckets),
                                         dtype=grad_dtype, device=dev)
            if not isinstance(emulate_comm, bool):
                self._emu_gbps = float(emulate_comm)
                if self._emu_gbps <= 0:
                    raise ValueError("emulate_comm bus bandwidth must be > 0 GB/s")
        # the optimizer runs in two ranges: everything but the last bucket as soon as those
        # buckets are reduced, then the last bucket — whose all-reduce (it is ready only at the
        # end of backward) overlaps the first range's AdamW instead of preceding all of it
        self.split_optimizer = split_optimizer
        self.opt_overlap = ((int(_OPT_OVERLAP) if _OPT_OVERLAP is not None
                             else (2 if self.world == 1 else 0))
                            if dev.type == "cuda" else 0)
        self._opt_stream = None
        self._opt_issued = 0          # head-bucket AdamW ranges issued in this step's backward
        self._in_step = False         # only step() (which joins the optimizer stream) overlaps
        self.side_stream_checks = []  # warm-up concurrency re-checks (_recheck_side_streams)
        self.timeline = False       # record comm events per bucket (comm_tail_report)
        self._tl = None
        self.step_count = 0

    def _setup_auto(self, comm: Comm, dev) -> None:
        """``allreduce="auto"``: every bucket on a probed (concurrency-checked) comm stream —
        the registered in-place IPC all-reduce for buckets up to the node-calibrated ``reg_max``
        (where it beat RCCL on rank-max time, ``CustomAllReduce.calibrate``), our native RCCL
        engine for the rest. ProcessGroupNCCL (whose internal pool stream may share the compute
        stream's hardware queue, parallel/streams.py) is only the last resort when the native
        engine cannot be created (e.g. ranks sharing one GPU). Per-bucket choice: ``bucket_paths``."""
        from .custom_allreduce import get_custom_allreduce

        self._comm_stream = concurrent_stream(dev, "ddp_comm", 0)
        car = get_custom_allreduce(comm)
        reg_max = int(getattr(car, "reg_max", 0) or 0) if car is not None else 0
        need_native = False
        for b in self.buckets:
            buf = self.flat_grad[b.start:b.end]
            nbytes = buf.numel() * buf.element_size()
            if (car is not None and car.reg_healthy and nbytes <= reg_max
                    and car.supports_registered(buf)):
                self._bucket_reg[b.idx] = car.register(buf)     # collective, same order
            else:
                need_native = True
        if self._bucket_reg:
            self._car = car
        if need_native:
            from .rccl_native import get_native

            try:
                self._native = get_native(comm)     # collective; failure agreed on every rank
            except RuntimeError as e:
                if comm.rank == 0:
                    print(f"[ddp auto] native RCCL engine unavailable ({e}); large buckets use "
                          "the process group", flush=True)

    def bucket_paths(self) -> Dict[int, str]:
        """Which all-reduce each bucket takes (result JSONs): ``custom_reg`` (registered IPC,
        in place), ``custom`` (IPC via staging), ``native`` (our RCCL engine on the comm
        stream), ``rccl`` (ProcessGroupNCCL), ``emulated`` or ``none`` (world 1)."""
        out = {}
        for b in self.buckets:
            buf = self.flat_grad[b.start:b.end]
            if self._emu_zero is not None:
                out[b.idx] = "emulated"
            elif self.world == 1:
                out[b.idx] = "none"
            elif b.idx in self._bucket_reg:
                out[b.idx] = "custom_reg"
            elif (self.allreduce == "custom" and self._car is not None and self._car.healthy
                  and self._car.supports(buf)):
                out[b.idx] = "custom"
            elif self._native is not None:
                out[b.idx] = "native"
            else:
                out[b.idx] = "rccl"
        return out

    # ------------------------------------------------------------------ hooks for subclasses
    def _bucket_align(self) -> int:
        return _ALIGN

    def _init_optimizer(self, lr, betas, weight_decay) -> None:
        self.master = self.flat_param.float()
        self.opt = FlatAdamW(self.master, lr=lr, betas=betas, weight_decay=weight_decay)

    def _optimizer_step(self, ranges=None, advance: bool = True) -> None:
        self.opt.step(self.flat_grad, working_bf16=self.flat_param, grad_scale=1.0 / self.world,
                      ranges=ranges, advance=advance)

    # ------------------------------------------------------------------ buckets
    def _add_bucket(self, start: int, end: int, params) -> None:
        b = _Bucket(len(self.buckets), start, end, list(params))
        for p in params:
            self._bucket_of[id(p)] = b
        self.buckets.append(b)

    def _reset(self) -> None:
        for b in self.buckets:
            b.ready, b.launched, b.work = 0, False, None
        self._next = 0
        self._opt_issued = 0
        for b in self.buckets:
            b.opt_done = False
        self._seen.clear()
        for p in self._params:          # per-step use counters of multi-use gradient sinks
            if getattr(p, "_dlbb_sink_count", 0):
                p._dlbb_sink_count = 0

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        # a param is counted once per step: a gradient-sink param reports itself from inside its
        # backward, and autograd may still run its post-accumulate hook (with no gradient)
        if id(p) in self._seen:
            return
        self._seen.add(id(p))
        b = self._bucket_of[id(p)]
        b.ready += 1
        if self.overlap and b.ready == len(b.params):
            self._launch_ready()

    def _launch_ready(self) -> None:
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if b.ready < len(b.params):
                return
            self._launch(b)
            self._next += 1
            self._maybe_opt_bucket(b)

    def _maybe_opt_bucket(self, b: _Bucket) -> None:
        """Overlapped split optimizer: AdamW of head bucket ``b`` on the optimizer stream, ordered
        after everything that produced or reads the bucket — the main stream up to now (its
        dgrads read these weights before the sinks report them ready, ops/linear_fn.py), the
        weight-gradient side streams, and the bucket's all-reduce. The first range of the step
        advances the AdamW step count; the tail bucket waits for this stream in ``step``."""
        if (not self.opt_overlap or not self._in_step or b.idx == len(self.buckets) - 1
                or not self._split_optimizer_ok()):
            return
        os_ = self._get_opt_stream()
        fork(os_)
        self._wait_wgrad(os_)
        with torch.cuda.stream(os_):
            self._wait_bucket(b)
            self._optimizer_step(ranges=[(b.start, b.end)], advance=self._opt_issued == 0)
        self._opt_issued += 1
        b.opt_done = True

    def recheck_side_streams(self) -> None:
        """Public form of the re-check (no-op without side streams, under CU-masked streams or
        during a capture); runners call it once after their warm-up steps."""
        if ((self._wgrad_stream is not None or self._comm_stream is not None)
                and not torch.cuda.is_current_stream_capturing()):
            self._recheck_side_streams()

    def _recheck_side_streams(self) -> None:
        """Warm-up check (once after a runner's warm-up steps, never inside the timed loop) that
        every weight-gradient stream still runs beside the stream the step runs on. A run whose compute stream waited, after every forked-from
        kernel, for exactly the side stream's weight-gradient + reduce kernels — the in-order
        execution of two streams sharing one hardware queue — took 19-19.6 ms instead of
        17.3-18 (profiles/r05_step/SUMMARY.md §12); a serialised side stream is replaced by a
        fresh one verified against the current compute stream."""
        dev = self.flat_grad.device
        cur = torch.cuda.current_stream(dev)
        bad = [i for i, ws in enumerate(self._wgrad_streams) if not runs_concurrently(cur, ws, dev)]
        rec = {"step": self.step_count, "serialised": len(bad)}
        if self._comm_stream is not None and not runs_concurrently(cur, self._comm_stream, dev):
            # the bucket reductions' stream (IPC / native RCCL / emulated): same check
            self._comm_stream = concurrent_stream(dev, f"ddp_comm_s{self.step_count}",
                                                  0, ref=cur)
            rec["comm_replaced"] = True
        if bad:
            new = list(self._wgrad_streams)
            for i in bad:
                new[i] = concurrent_stream(dev, f"ddp_wgrad_s{self.step_count}_{i}", 0, ref=cur)
            remap = {i: new[i] for i in bad}
            for q in self._params:
                old = getattr(q, "_dlbb_grad_stream", None)
                if old is None:
                    continue
                for i in bad:
                    if old is self._wgrad_streams[i]:
                        q._dlbb_grad_stream = remap[i]
            if self._opt_stream is not None and any(self._opt_stream is self._wgrad_streams[i]
                                                    for i in bad):
                self._opt_stream = None
            self._wgrad_streams = new
            self._wgrad_stream = new[0]
            rec["replaced"] = bad
            rec["now_concurrent"] = all(runs_concurrently(cur, ws, dev) for ws in new)
        self.side_stream_checks.append(rec)

    def _get_opt_stream(self):
        if self._opt_stream is None:
            self._opt_stream = (self._wgrad_stream if self.opt_overlap == 2
                                and self._wgrad_stream is not None
                                else concurrent_stream(self.flat_grad.device, "ddp_opt"))
        return self._opt_stream

    def _launch(self, b: _Bucket) -> None:
        b.launched = True
        if self.mode == "flatten":
            # autograd allocates fresh .grad tensors each step: the table is keyed by their
            # addresses (the caching allocator usually hands back the same blocks, so it is
            # rebuilt only when a block moved)
            key = tuple(p.grad.data_ptr() for p in b.params)
            if b.table is None or b.table_key != key:
                pairs = [(p.grad.reshape(-1), self.flat_grad[self._offsets[id(p)]:
                                                              self._offsets[id(p)] + p.numel()])
                         for p in b.params]
                # fp32 buckets (mode="flatten", grad_dtype=fp32): the flatten pass also casts
                b.table = (ChunkTable(pairs) if self.flat_grad.dtype == b.params[0].grad.dtype
                           else ScaleTable(pairs, 1.0))
                b.table_key = key
            b.table.run()
        if self._emu_zero is not None:
            buf = self.flat_grad[b.start:b.end]
            cs = self._comm_stream
            fork(cs)
            with torch.cuda.stream(cs):
                self._tl_mark(b, "start", cs)
                reduce_sum([buf, self._emu_zero[:buf.numel()]], out=buf,
                           nblocks=self.comm_blocks)
                if self._emu_gbps is not None:
                    P = self._emu_world
                    nbytes = buf.numel() * buf.element_size()
                    ns = int(nbytes * 2.0 * (P - 1) / P / self._emu_gbps)   # bytes / (GB/s) = ns
                    spin_ns(ns, self.comm_blocks or 32)
                self._tl_mark(b, "end", cs)
            self._mark_done(b, cs)
            b.work = "stream"
            return
        if self.world == 1:
            return
        buf = self.flat_grad[b.start:b.end]
        ws = self._wgrad_stream
        if b.idx in self._bucket_reg:
            cs = self._comm_stream
            fork(cs)
            if ws is not None:
                self._wait_wgrad(cs)
            with torch.cuda.stream(cs):
                self._tl_mark(b, "start", cs)
                self._car.all_reduce_registered(buf, self._bucket_reg[b.idx],
                                                nblocks=self.comm_blocks)
                self._tl_mark(b, "end", cs)
            self._mark_done(b, cs)
            b.work = "stream"
        elif (self.allreduce == "custom" and self._car is not None and self._car.healthy
              and self._car.supports(buf)):
            cs = self._comm_stream
            fork(cs)
            if ws is not None:
                self._wait_wgrad(cs)
            with torch.cuda.stream(cs):
                self._tl_mark(b, "start", cs)
                self._car.all_reduce_(buf, nblocks=self.comm_blocks)
                self._tl_mark(b, "end", cs)
            self._mark_done(b, cs)
            b.work = "stream"
        elif self._native is not None:
            # our RCCL communicator on the dedicated comm stream, ordered after the
            # producing backward kernels; finish() joins the stream
            cs = self._comm_stream
            fork(cs)
            if ws is not None:
                self._wait_wgrad(cs)
            self._tl_mark(b, "start", cs)
            self._native.enqueue("allreduce", buf, buf, buf.numel(), stream=cs.cuda_stream)
            self._tl_mark(b, "end", cs)
            self._mark_done(b, cs)
            b.work = "stream"
        elif ws is not None:
            # ProcessGroupNCCL orders its stream after the CURRENT stream: issue from the side
            # stream once it has joined the main one (covers both producers)
            ws.wait_stream(torch.cuda.current_stream(buf.device))
            for other in self._wgrad_streams[1:]:
                ws.wait_stream(other)
            with torch.cuda.stream(ws):
                b.work = dist.all_reduce(buf, async_op=True)
        else:
            b.work = dist.all_reduce(buf, async_op=True)

    def _wait_wgrad(self, stream) -> None:
        """Order ``stream`` after every weight-gradient side stream (not after itself: a
        stream waiting on its own event inside a HIP-graph capture crashes capture_end)."""
        for ws in self._wgrad_streams:
            if ws != stream:
                fork(stream, ws)

    def _mark_done(self, b: _Bucket, cs) -> None:
        """Per-bucket completion event on the comm stream (waited per bucket by the split
        optimizer; a stream-wide wait would also wait for later buckets)."""
        ev = b.done_event
        if ev is None:
            ev = b.done_event = torch.cuda.Event()
        ev.record(cs)

    def _tl_mark(self, b: _Bucket, what: str, stream) -> None:
        if self._tl is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        self._tl["buckets"].setdefault(b.idx, {})[what] = ev

    def _wait_bucket(self, b: _Bucket) -> None:
        if b.work == "stream":
            cur = torch.cuda.current_stream(self.flat_grad.device)
            if b.done_event is not None:
                cur.wait_event(b.done_event)
            else:
                cur.wait_stream(self._comm_stream)
        elif b.work is not None:
            b.work.wait()

    def _launch_rest(self) -> None:
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            self._launch(b)
            self._next += 1
            self._maybe_opt_bucket(b)

    def finish(self) -> None:
        """Launch what backward did not (e.g. overlap off), then wait every bucket."""
        self._launch_rest()
        for b in self.buckets:
            self._wait_bucket(b)
        if self._wgrad_stream is not None:      # side-stream weight gradients (and copies)
            self._wait_wgrad(torch.cuda.current_stream(self.flat_grad.device))

    def check_comm_errors(self) -> None:
        """Collective: raise on every rank if an IPC all-reduce of any rank timed out since the
        last check (its spin wait gave up: the reduced gradients are partial). One small
        synchronous read per rank + one object all-gather: call it every few steps and at the
        end of a run, outside timed regions (a timeout must never pass silently)."""
        if self._car is not None:
            self._car.raise_if_error()

    # ------------------------------------------------------------------ step
    def zero_grad(self) -> None:
        if self.mode == "view":
            self.flat_grad.zero_()
            for p in self._params:      # sink writers may store instead of accumulate once
                if hasattr(p, "_dlbb_grad_sink"):
                    p._dlbb_grad_fresh = True
        else:
            for p in self._params:
                p.grad = None

    def step(self, idx: torch.Tensor, targets: torch.Tensor, sync_loss: bool = True):
        """One full training step: forward, backward (+ overlapped all-reduce), AdamW."""
        self.zero_grad()
        self._reset()
        self._in_step = True
        if self.timeline and not torch.cuda.is_current_stream_capturing():
            self._tl = {"buckets": {}}
        with tracing.range("fwd"):
            loss = self.model(idx, targets)
        with tracing.range("bwd+overlapped_grad_sync"):
            mark_unit_upstream(loss)        # loss.backward(): the fused loss skips its scaling
            loss.backward()
        if self._tl is not None:
            self._tl["bwd_end"] = torch.cuda.Event(enable_timing=True)
            self._tl["bwd_end"].record(torch.cuda.current_stream(self.flat_grad.device))
        self.step_count += 1
        if self._split_optimizer_ok():
            with tracing.range("grad_sync_tail+optimizer"):
                self._launch_rest()
                head, tail = self.buckets[:-1], self.buckets[-1]
                cur = (torch.cuda.current_stream(self.flat_grad.device)
                       if self.flat_grad.is_cuda else None)
                if self._opt_issued:
                    # AdamW ranges already queued on the optimizer stream during backward
                    fork(cur, self._opt_stream)
                todo = [b for b in head if not b.opt_done]
                for b in todo:
                    self._wait_bucket(b)
                if self._wgrad_stream is not None:
                    self._wait_wgrad(cur)
                adv = self._opt_issued == 0
                if todo:
                    self._optimizer_step(
                        ranges=[(0, tail.start)] if len(todo) == len(head)
                        else [(b.start, b.end) for b in todo], advance=adv)
                    adv = False
                self._wait_bucket(tail)
                self._optimizer_step(ranges=[(tail.start, self.numel)], advance=adv)
        else:
            with tracing.range("grad_sync_tail"):
                self.finish()
            with tracing.range("optimizer"):
                self._optimizer_step()
        self._in_step = False
        if self._tl is not None:
            self._tl["opt_end"] = torch.cuda.Event(enable_timing=True)
            self._tl["opt_end"].record(torch.cuda.current_stream(self.flat_grad.device))
            self._tl_last, self._tl = self._tl, None
        return float(loss.item()) if sync_loss else loss.detach()

    def _split_optimizer_ok(self) -> bool:
        return (self.split_optimizer and len(self.buckets) > 1 and self.mode == "view"
                and type(self)._optimizer_step is FlatParamTrainer._optimizer_step)

    def comm_tail_report(self) -> Optional[dict]:
        """For the last step run with ``timeline = True`` (stream-issued reductions: custom,
        native, emulated): each bucket's comm start / end relative to the end of backward, the
        bytes whose reduction STARTED after backward ended, and the exposed comm time (last
        reduction end minus backward end; 0 when everything finished under backward)."""
        tl = getattr(self, "_tl_last", None)
        if not tl or "bwd_end" not in tl:
            return None
        torch.cuda.synchronize(self.flat_grad.device)
        ref = tl["bwd_end"]
        rows, after, last_end = [], 0, float("-inf")
        esz = self.flat_grad.element_size()
        for b in self.buckets:
            e = tl["buckets"].get(b.idx)
            if not e or "start" not in e or "end" not in e:
                continue
            st, en = ref.elapsed_time(e["start"]), ref.elapsed_time(e["end"])
            nbytes = (b.end - b.start) * esz
            rows.append({"bucket": b.idx, "bytes": nbytes, "start_ms": round(st, 4),
                         "end_ms": round(en, 4)})
            if st >= 0:
                after += nbytes
            last_end = max(last_end, en)
        return {"buckets": rows, "bytes_reduced_after_backward": after,
                "exposed_comm_ms": round(max(0.0, last_end), 4) if rows else None,
                "optimizer_end_ms": round(ref.elapsed_time(tl["opt_end"]), 4)
                if "opt_end" in tl else None}

    # ------------------------------------------------------------------ HIP graph
    def capture_step(self, idx: torch.Tensor, targets: torch.Tensor):
        """Capture one whole training step (forward, backward with its bucket reductions, AdamW)
        into a HIP graph and return ``replay(idx, targets) -> loss`` (a device tensor).

        Capturable when nothing in the step goes through ProcessGroupNCCL (its watchdog breaks
        capture on this stack): world 1, or bucket reductions on the native RCCL engine /
        the IPC kernel. The optimizer's step count moves to device memory. One eager step is run
        first (a real training step) to settle lazily created state; GEMM choices are already
        cached by earlier eager steps."""
        if self.world > 1 and self._native is None and self._car is None:
            raise RuntimeError("graph capture needs world 1 or allreduce='native'|'custom'")
        self.opt.enable_device_step()
        dev = self.flat_param.device
        static_idx, static_tgt = idx.clone(), targets.clone()
        cur = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self.step(static_idx, static_tgt, sync_loss=False)
        cur.wait_stream(side)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        dot = os.environ.get("DLBB_GRAPH_DOT")   # diagnostics: dump the captured topology
        if dot:
            graph.enable_debug_mode()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            static_loss = self.step(static_idx, static_tgt, sync_loss=False)
        if dot:
            graph.debug_dump(dot)
        # capture recorded the step without running it: undo the host-side bookkeeping
        self.step_count -= 1
        self.opt.t -= 1

        def replay(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
            static_idx.copy_(x)
            static_tgt.copy_(y)
            graph.replay()
            self.step_count += 1
            self.opt.t += 1
            return static_loss

        replay.graph = graph
        return replay

    # ------------------------------------------------------------------ checkpoint / resume
    # The reference has no checkpointing. Here the optimizer state is three flat
    # fp32 buffers (+ the step counter), so a checkpoint is one safetensors file per state owner:
    # rank 0 for replicated DDP, every rank for ZeRO shards. Layout = the flat bucket layout,
    # which is a pure function of the model and (bucket_mb, world) — checked on load.
    def _replicated_state(self) -> bool:
        return True

    def layout_signature(self) -> Dict:
        return {"kind": type(self).__name__, "numel": int(self.numel),
                "master_numel": int(self.master.numel()), "world": int(self.world),
                "buckets": [[b.start, b.end] for b in self.buckets]}

    def state_tensors(self) -> Dict[str, torch.Tensor]:
        return {"master": self.master, "exp_avg": self.opt.m, "exp_avg_sq": self.opt.v}

    def save_checkpoint(self, path: str) -> None:
        from safetensors.torch import save_file

        rank = self.comm.rank if self.comm is not None else 0
        owner = (not self._replicated_state()) or rank == 0
        meta = {**self.layout_signature(), "step": self.step_count, "adam_t": self.opt.t}
        if owner:
            os.makedirs(path, exist_ok=True)
            name = os.path.join(path, f"rank{rank:05d}.safetensors")
            tmp = name + ".tmp"
            save_file({k: v.detach().contiguous().cpu() for k, v in self.state_tensors().items()},
                      tmp, metadata={"meta": json.dumps(meta)})
            os.replace(tmp, name)
            if rank == 0:
                with open(os.path.join(path, "meta.json.tmp"), "w") as f:
                    json.dump(meta, f, indent=2)
                os.replace(os.path.join(path, "meta.json.tmp"), os.path.join(path, "meta.json"))
        if self.comm is not None:
            self.comm.barrier()

    @torch.no_grad()
    def load_checkpoint(self, path: str) -> None:
        from safetensors import safe_open

        rank = self.comm.rank if self.comm is not None else 0
        src_rank = 0 if self._replicated_state() else rank
        name = os.path.join(path, f"rank{src_rank:05d}.safetensors")
        with safe_open(name, framework="pt", device="cpu") as f:
            meta = json.loads(f.metadata()["meta"])
            want = self.layout_signature()
            for k in ("kind", "numel", "master_numel", "buckets"):
                if meta[k] != want[k]:
                    raise ValueError(f"checkpoint {name}: {k} mismatch ({meta[k]} != {want[k]})")
            if not self._replicated_state() and meta["world"] != want["world"]:
                raise ValueError("sharded checkpoint written with world "
                                 f"{meta['world']}, loading with {want['world']}")
            for k, t in self.state_tensors().items():
                t.copy_(f.get_tensor(k).to(t.device))
        self.opt.t = int(meta["adam_t"])
        if self.opt.t_dev is not None:         # HIP-graph mode reads the device counter
            self.opt.t_dev.fill_(self.opt.t)
        self.step_count = int(meta["step"])
        self._refresh_params()

    def _refresh_params(self) -> None:
        self.flat_param.copy_(self.master.to(torch.bfloat16))

    def close(self) -> None:
        """Remove hooks / sink attributes and release the buckets' IPC registrations
        (collective when any bucket is registered: call on every rank)."""
        if self._bucket_reg and self._car is not None:
            torch.cuda.synchronize(self.flat_grad.device)
            for idx in sorted(self._bucket_reg):
                self._car.deregister(self._bucket_reg[idx])
            self._bucket_reg = {}
        for h in self._hooks:
            h.remove()
        for p in self._params:
            for attr in ("_dlbb_grad_sink", "_dlbb_grad_stream", "_dlbb_sink_count",
                         "_dlbb_grad_fresh", "_dlbb_grad_event"):
                if hasattr(p, attr):
                    delattr(p, attr)
