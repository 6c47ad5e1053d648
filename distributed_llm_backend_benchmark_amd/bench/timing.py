"""Timing loops for one collective.

Reference methodology (``collectives/1d/openmpi.py:60-65``, ``collectives/1d/dsccl.py:61-67``):
barrier → host clock → blocking call → host clock, per iteration. On a GPU a collective call
only enqueues work, so we keep the per-iteration barrier and time with HIP events on the
caller's stream around the call (device time, the RCCL kernel including any wait for late
peers), synchronising after each iteration; the host ``perf_counter`` interval (launch +
execution + sync) is recorded alongside. Every rank's ``[iter]`` list is gathered to rank 0
as ``[rank][iter]`` (reference ``collectives/1d/openmpi.py:270``).

``batched`` mode is the nccl-tests methodology: ``iters`` back-to-back calls between one
event pair (optionally replayed from a captured HIP graph), reporting the mean per call.
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from ..parallel.collectives import CollectiveOp
from ..parallel.comm import Comm


@dataclass
class TimingResult:
    timings: List[float]                     # seconds, this rank, per iteration
    host_timings: List[float] = field(default_factory=list)
    timing_method: str = "hip_event"
    batched_mean_s: Optional[float] = None   # nccl-tests style mean per call
    batched_method: Optional[str] = None


def _warm(comm: Comm, op: CollectiveOp, warmup: int) -> None:
    for _ in range(warmup):
        op.reset()
        comm.sync()
        comm.barrier()
        op.run()
    comm.sync()


def time_per_iteration(comm: Comm, op: CollectiveOp, iters: int, warmup: int,
                       method: str = "auto") -> TimingResult:
    """Reference-compatible ``[iter]`` timings for this rank."""
    gpu = comm.is_gpu
    if method == "auto":
        method = "hip_event" if gpu else "host_perf_counter"
    _warm(comm, op, warmup)
    times: List[float] = []
    host: List[float] = []
    if gpu and method == "hip_event":
        stream = torch.cuda.current_stream(comm.device)
        starts = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(iters)]
        for i in range(iters):
            op.reset()
            comm.sync()
            comm.barrier()
            t0 = time.perf_counter()
            starts[i].record(stream)
            op.run()
            ends[i].record(stream)
            stream.synchronize()
            host.append(time.perf_counter() - t0)
        times = [s.elapsed_time(e) * 1e-3 for s, e in zip(starts, ends)]
    else:
        for _ in range(iters):
            op.reset()
            comm.sync()
            comm.barrier()
            t0 = time.perf_counter()
            op.run()
            comm.sync()
            times.append(time.perf_counter() - t0)
        host = list(times)
        method = "host_perf_counter"
    return TimingResult(timings=times, host_timings=host, timing_method=method)


def time_batched(comm: Comm, op: CollectiveOp, iters: int, warmup: int,
                 graph: bool = False) -> float:
    """Mean seconds per call over ``iters`` back-to-back calls (nccl-tests style)."""
    _warm(comm, op, max(1, warmup))
    if not comm.is_gpu:
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            op.run()
        return (time.perf_counter() - t0) / iters
    stream = torch.cuda.current_stream(comm.device)
    runner = None
    if graph and graph_safe(op):
        runner = _capture(comm, op, iters)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    comm.sync()
    comm.barrier()
    s.record(stream)
    if runner is not None:
        runner.replay()
    else:
        for _ in range(iters):
            op.run()
    e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) * 1e-3 / iters


def graph_safe(op: CollectiveOp) -> bool:
    """HIP-graph capture is used for ops that do not go through torch's ProcessGroupNCCL: the
    IPC xGMI all-reduce (pure HIP kernels) and the native RCCL engine (RCCL enqueued directly on
    the capturing stream). RCCL collectives issued through ProcessGroupNCCL race its watchdog
    thread's event queries on ROCm 7.0 / torch 2.10 (hipErrorCapturedEvent aborts the process),
    so they are timed back to back instead."""
    return getattr(op, "impl", None) in ("custom", "native")


def _capture(comm: Comm, op: CollectiveOp, iters: int):
    """Capture ``iters`` calls into one HIP graph (launch overhead amortised)."""
    side = torch.cuda.Stream(comm.device)
    side.wait_stream(torch.cuda.current_stream(comm.device))
    with torch.cuda.stream(side):
        op.run()  # warm caches / lazily created communicators outside capture
    torch.cuda.current_stream(comm.device).wait_stream(side)
    comm.sync()
    g = torch.cuda.CUDAGraph()
    # thread_local: ProcessGroupNCCL's watchdog thread keeps querying events while we capture
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(iters):
            op.run()
    comm.sync()
    g.replay()  # one untimed replay
    comm.sync()
    return g
