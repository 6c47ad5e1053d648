"""The roofline guard in the sweep writer and in the stats stage: a P=1
1 GiB all-reduce "timed" at 14 us (an in-place call that enqueued nothing — the committed
round-1 dataset held such rows at 77 TB/s) is refused by both, never written as a result."""

import json
import os

from distributed_llm_backend_benchmark_amd.bench import sweep
from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
from distributed_llm_backend_benchmark_amd.stats import stats1d, stats3d

GIB = 1 << 30


def _fake_bench_one(comm, op_name, data, warmup, iters, timing, batched, graph, validate, seed,
                    op_opts, label=""):
    return {"op_impl": "rccl", "timings": [[14e-6] * iters], "host_timings": [[20e-6] * iters],
            "timing_method": "hip_event", "message_bytes": GIB, "num_elements": GIB // 2}


def test_sweep_writer_refuses_below_roofline(tmp_path, monkeypatch):
    monkeypatch.setattr(sweep, "_bench_one", _fake_bench_one)
    comm = init_distributed("gloo")
    try:
        out = tmp_path / "1d"
        written = sweep.run_1d_sweep(comm, ops=["allreduce"], sizes={"1GB": 256}, iters=5,
                                     warmup=1, output_dir=str(out), impl_name="rccl")
        assert written == []
        err = json.load(open(out / "rccl_allreduce_ranks1_1GB.error.json"))
        assert err["invalid"] == "below_roofline" and "roofline" in err["error"]
        assert not (out / "rccl_allreduce_ranks1_1GB.json").exists()
        out3 = tmp_path / "3d"
        written = sweep.run_3d_sweep(comm, ops=["allgather"], batch_sizes=[1], seq_lengths=[2],
                                     hidden_dims=[8], iters=5, warmup=1, output_dir=str(out3),
                                     impl_name="rccl")
        assert written == [] and any(f.endswith(".error.json") for f in os.listdir(out3))
    finally:
        comm.destroy()


def _raw_1d(n_elems, t, ranks=1, op="allreduce", **kw):
    return dict({"implementation": "rccl", "operation": op, "num_ranks": ranks,
                 "data_size_name": "x", "num_elements": n_elems, "dtype": "bfloat16",
                 "bytes": n_elems * 2, "warmup_iterations": 1, "measurement_iterations": 3,
                 "timings": [[t] * 3] * ranks}, **kw)


def test_stats_refuse_impossible_rows(tmp_path):
    raw = tmp_path / "raw"
    raw.mkdir()
    json.dump(_raw_1d(GIB // 2, 14e-6), open(raw / "rccl_allreduce_ranks1_1GB.json", "w"))
    json.dump(_raw_1d(GIB // 2, 0.7e-3), open(raw / "rccl_allreduce_ranks1_ok.json", "w"))
    json.dump(_raw_1d(256, 5e-6, invalid="wrong result"), open(raw / "rccl_bad.json", "w"))
    rows = stats1d.process_directory(str(raw), str(tmp_path / "st"), verbose=False)
    assert [r["median_time_us"] for r in rows] == [700.0]
    d3 = tmp_path / "raw3"
    d3.mkdir()
    rec = {"implementation": "rccl", "operation": "allreduce", "num_ranks": 1,
           "tensor_shape": {"batch": 32, "seq_len": 8192, "hidden_dim": 4096},
           "num_elements": 32 * 8192 * 4096, "tensor_size_bytes": 2 * GIB,
           "tensor_size_mb": 2048.0, "dtype": "bfloat16", "timings": [[13e-6] * 3]}
    json.dump(rec, open(d3 / "a.json", "w"))
    assert stats3d.process_directory(str(d3), str(tmp_path / "st3"), "rccl", verbose=False) == []


def test_reference_rows_pass_the_guard():
    """The reference's own CPU data (P=2..16) is far above any roofline: none is refused."""
    import glob

    ref = os.path.join(os.path.dirname(__file__), "fixtures", "reference")
    files = [f for f in glob.glob(os.path.join(ref, "**", "*.json"), recursive=True)]
    seen = 0
    for f in files:
        d = json.load(open(f))
        if "timings" in d and "operation" in d and "num_ranks" in d and (
                "num_elements" in d):
            seen += 1
            assert stats1d.refused(d) is None, f
    assert seen > 0


def test_no_committed_csv_row_beats_the_roofline():
    """every committed stats row (results/**) is physically possible. The
    virtual-rank dataset (results/vr_custom: W ranks on ONE GPU) is bounded by the W ranks'
    combined traffic on that device (colocated)."""
    import csv
    import glob

    from distributed_llm_backend_benchmark_amd.stats.bandwidth import (KNOWN_OPS,
                                                                        roofline_violation)

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = 0
    for path in glob.glob(os.path.join(repo, "results", "**", "*_ext.csv"), recursive=True):
        coloc = "vr_custom" in path
        for r in csv.DictReader(open(path)):
            op = r["operation"]
            if op not in KNOWN_OPS:
                continue
            if "median_time_ms" in r:
                t = float(r["median_time_ms"]) / 1e3
                nbytes = float(r.get("wire_bytes") or r["tensor_size_bytes"])
            else:
                t = float(r["median_time_us"]) / 1e6
                nbytes = float(r["bytes"])
            why = roofline_violation(op, nbytes, t, int(r["num_ranks"]), coloc)
            assert why is None, (path, why)
            rows += 1
    assert rows > 100
