"""bench.py's honesty guard: a timing below the traffic-based roofline (an empty call, or one
that missed its work) is rejected, for the P = 1 copy and per op at P > 1."""

import importlib.util
import os

import pytest

from distributed_llm_backend_benchmark_amd.stats import bandwidth as bw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


MIB = 1 << 20


@pytest.mark.parametrize("op,nbytes,P,seconds,ok", [
    # P = 1: the out-of-place copy moves 2x the message (read + write)
    ("allreduce", 64 * MIB, 1, 20.4e-6, True),          # BENCH_r02: 6.6 TB/s of traffic, on die
    ("allreduce", 64 * MIB, 1, 5e-6, False),            # an empty call's host overhead
    ("allreduce", 1 << 30, 1, 449e-6, True),            # BENCH_r02 sweep: 4.8 TB/s
    # algBW 7.2 TB/s passed round 2's algBW-vs-8 TB/s guard; the copy's traffic is 14.3 TB/s
    ("allreduce", 1 << 30, 1, 150e-6, False),
    # P > 1: the xGMI receive bound (bytes (P-1)/P over P-1 links)
    ("allreduce", 64 * MIB, 8, 400e-6, True),           # busBW 294 GB/s
    ("allreduce", 64 * MIB, 8, 30e-6, False),           # busBW 3.9 TB/s: impossible over xGMI
    ("allgather", 64 * MIB, 8, 0.5e-3, True),
    ("allgather", 64 * MIB, 8, 0.2e-3, False),          # 7 x 64 MiB in 0.2 ms
    ("reduce_scatter", 64 * MIB, 4, 10e-6, False),
    ("alltoall", 64 * MIB, 2, 1e-3, True),
    ("allreduce", 512, 2, 9e-6, True),                  # small messages: latency, never rejected
])
def test_too_fast_rejects_impossible_timings(op, nbytes, P, seconds, ok):
    bench = _bench()
    why = bench.too_fast(op, nbytes, seconds, P)
    assert (why is None) == ok, why
    assert (bw.roofline_violation(op, nbytes, seconds, P) is None) == ok


def test_min_seconds_monotone_in_bytes_and_known_ops():
    for op in ("allreduce", "allgather", "reduce_scatter", "alltoall", "broadcast", "reduce",
               "gather", "scatter", "sendrecv", "alltoall_moe"):
        for P in (1, 2, 8):
            a = bw.min_seconds(op, MIB, P)
            b = bw.min_seconds(op, 64 * MIB, P)
            assert 0 < a < b
    with pytest.raises(KeyError):
        bw.min_seconds("nonsense", MIB, 2)


def test_colocated_ranks_bound_is_device_memory_not_links():
    """Ranks sharing one GPU (the two-rank rehearsal on a one-GPU box) cross no xGMI link: a
    64 MiB all-reduce at P=2 in 75 us (~4 TB/s of combined traffic) is possible there, while
    across two GPUs it would beat the link peak."""
    nbytes = 64 * MIB
    assert bw.roofline_violation("allreduce", nbytes, 75e-6, 2) is not None
    assert bw.roofline_violation("allreduce", nbytes, 75e-6, 2, colocated=True) is None
    # an empty call is still caught
    assert bw.roofline_violation("allreduce", nbytes, 2e-6, 2, colocated=True) is not None
    assert bw.min_seconds("allreduce", nbytes, 2, colocated=True) > bw.min_seconds(
        "allreduce", nbytes, 1)
