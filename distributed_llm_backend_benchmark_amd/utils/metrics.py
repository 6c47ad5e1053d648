"""Metrics collection and timing.

``MetricsCollector`` keeps the reference's field names (``utils.py:17-70``: init/warmup/forward
times and a summary with mean/std/min/max/median/p95/p99) so result JSONs stay comparable.

``Timer`` differs from the reference's ``time.time()`` bracket (``utils.py:73-87``): on a GPU the
forward is asynchronous, so the timer synchronises the current HIP stream on exit (and
optionally records HIP events) — otherwise it would time kernel *launches*, not execution.
"""

from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence

import numpy as np


def summarize(values: Sequence[float], prefix: str = "") -> Dict[str, float]:
    arr = np.asarray(values, dtype=np.float64)
    if arr.size == 0:
        return {}
    return {
        f"{prefix}mean": float(np.mean(arr)),
        f"{prefix}std": float(np.std(arr)),
        f"{prefix}min": float(np.min(arr)),
        f"{prefix}max": float(np.max(arr)),
        f"{prefix}median": float(np.median(arr)),
        f"{prefix}p95": float(np.percentile(arr, 95)),
        f"{prefix}p99": float(np.percentile(arr, 99)),
    }


class MetricsCollector:
    """Per-rank experiment metrics (reference ``utils.py:17-70``)."""

    def __init__(self, rank: int, world_size: int):
        self.rank = rank
        self.world_size = world_size
        self.metrics: Dict[str, object] = {
            "init_time": None,
            "warmup_times": [],
            "forward_times": [],
        }

    def record_init_time(self, elapsed: float) -> None:
        self.metrics["init_time"] = elapsed

    def record_warmup_time(self, elapsed: float) -> None:
        self.metrics["warmup_times"].append(elapsed)

    def record_forward_time(self, elapsed: float) -> None:
        self.metrics["forward_times"].append(elapsed)

    def record(self, key: str, elapsed: float) -> None:
        self.metrics.setdefault(key, []).append(elapsed)

    def get_summary(self) -> Dict[str, object]:
        ft = self.metrics["forward_times"]
        s = {
            "rank": self.rank,
            "world_size": self.world_size,
            "init_time": self.metrics["init_time"],
            "num_iterations": len(ft),
        }
        s.update(summarize(ft, prefix="forward_"))
        return s

    def get_raw_metrics(self) -> Dict[str, object]:
        return self.metrics


class Timer:
    """Wall-clock context manager; with ``sync=True`` the current HIP stream is synchronised
    before reading the clock on exit so the interval covers device execution."""

    def __init__(self, sync: bool = False, device: Optional[object] = None):
        self.sync = sync
        self.device = device
        self.start_time: Optional[float] = None
        self.elapsed: Optional[float] = None

    def _sync(self) -> None:
        if self.sync:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize(self.device)

    def __enter__(self) -> "Timer":
        self._sync()
        self.start_time = time.perf_counter()
        return self

    def __exit__(self, *args) -> None:
        self._sync()
        self.elapsed = time.perf_counter() - self.start_time


class EventTimer:
    """HIP-event interval on a stream (device time, excludes host launch latency)."""

    def __init__(self, stream=None):
        import torch

        self.stream = stream
        self._s = torch.cuda.Event(enable_timing=True)
        self._e = torch.cuda.Event(enable_timing=True)

    def __enter__(self) -> "EventTimer":
        self._s.record(self.stream)
        return self

    def __exit__(self, *args) -> None:
        self._e.record(self.stream)

    def seconds(self) -> float:
        self._e.synchronize()
        return self._s.elapsed_time(self._e) * 1e-3


def print_summary(summary: Dict[str, object], backend_name: str, rank: int) -> None:
    """Reference ``utils.py:247-265``."""
    if rank != 0:
        return
    print("\n" + "=" * 60)
    print(f"RESULTS - {backend_name}")
    print("=" * 60)
    print(f"Initialization time: {summary['init_time']:.4f}s")
    print(f"Forward pass mean:   {summary['forward_mean']:.4f}s")
    print(f"Forward pass std:    {summary['forward_std']:.4f}s")
    print(f"Forward pass p95:    {summary['forward_p95']:.4f}s")
    print(f"Forward pass p99:    {summary['forward_p99']:.4f}s")
    print("=" * 60)


def rank_statistics(per_rank_means: List[float]) -> Dict[str, object]:
    """Variance / coefficient of variation across ranks (reference ``run_mpi.py:201-212``)."""
    arr = np.asarray(per_rank_means, dtype=np.float64)
    mean = float(np.mean(arr))
    return {
        "forward_mean_per_rank": arr.tolist(),
        "variance_across_ranks": float(np.var(arr)),
        "coefficient_of_variation": float(np.std(arr) / mean) if mean > 0 else 0.0,
    }


def gather_metrics_from_all_ranks(comm, local_summary: Dict[str, object]
                                  ) -> Optional[Dict[str, object]]:
    """Per-rank forward means (and p95s) to rank 0 with variance / CV.

    Reference ``utils.py:172-209`` (``dist.gather`` of float32 scalars; defined but never called
    there). Here it rides the job's process group through :class:`..parallel.comm.Comm`; returns
    the statistics on rank 0 and ``None`` elsewhere."""
    pairs = comm.all_gather_object((float(local_summary["forward_mean"]),
                                    float(local_summary.get("forward_p95", 0.0))))
    if comm.rank != 0:
        return None
    out = rank_statistics([m for m, _ in pairs])
    out["forward_p95_per_rank"] = [p for _, p in pairs]
    return out


def run_experiment(model, dataset, config: Dict[str, object], metrics: "MetricsCollector",
                   comm=None) -> "MetricsCollector":
    """Warmup + timed forwards (reference ``utils.py:212-244``). The reference times each
    forward with ``time.time()`` around an asynchronous call; here the timer synchronises the
    device (``Timer(sync=True)``), and with ``comm`` every timed forward is bracketed by
    barriers like ``run_mpi.py:177,183``."""
    ex = config["execution"]
    for _ in range(int(ex["warmup_iterations"])):
        batch = dataset.get_batch()
        with Timer(sync=True) as t:
            model(batch)
        metrics.record_warmup_time(t.elapsed)
    for _ in range(int(ex["benchmark_iterations"])):
        batch = dataset.get_batch()
        if comm is not None:
            comm.barrier()
        with Timer(sync=True) as t:
            model(batch)
        if comm is not None:
            comm.barrier()
        metrics.record_forward_time(t.elapsed)
    return metrics
