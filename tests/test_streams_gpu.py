"""Side streams verified to run beside the compute stream (parallel/streams.py)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_concurrent_stream_overlaps_compute_and_is_cached():
    from distributed_llm_backend_benchmark_amd.parallel import streams

    dev = torch.device("cuda", 0)
    cur = torch.cuda.current_stream(dev)
    a = streams.concurrent_stream(dev, "test_a")
    b = streams.concurrent_stream(dev, "test_b")
    assert a != cur and b != cur and a != b
    # the property the probe selected for, re-measured: a pair of spins takes ~one spin
    assert streams.runs_concurrently(cur, a, dev)
    assert streams.runs_concurrently(cur, b, dev)
    assert streams.runs_concurrently(a, b, dev)
    assert streams.concurrent_stream(dev, "test_a") is a


def test_same_stream_is_not_concurrent():
    """The probe can tell serialisation apart: one stream with itself runs in order."""
    from distributed_llm_backend_benchmark_amd.parallel import streams

    cur = torch.cuda.current_stream()
    assert not streams.runs_concurrently(cur, cur)
