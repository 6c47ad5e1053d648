"""Golden-schema tests: our stats over the reference's own result JSONs reproduce the reference's
per-file stats JSONs and CSV rows (fixtures copied from /root/reference/collectives/**; only
files whose committed stats were computed from the committed raw file — SURVEY §2.7 notes 113/512
1D files come from different runs)."""

import csv
import glob
import json
import os

import pytest

from conftest import FIXTURES
from distributed_llm_backend_benchmark_amd.stats import stats1d, stats3d
from distributed_llm_backend_benchmark_amd.stats.bandwidth import (algbw_gbps, bus_factor,
                                                                   busbw_gbps,
                                                                   legacy_bandwidth_gbps)

F1 = os.path.join(FIXTURES, "reference", "1d")
F3 = os.path.join(FIXTURES, "reference", "3d")


def _close(a, b, rel=1e-9):
    return abs(a - b) <= rel * max(1.0, abs(a), abs(b))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(F1, "results", "*.json"))))
def test_1d_stats_match_reference(path):
    ref = json.load(open(os.path.join(F1, "stats", os.path.basename(path)[:-5] + "_stats.json")))
    got = stats1d.stats_for_result(json.load(open(path)))
    for k in ("mean_time_us", "median_time_us", "min_time_us", "max_time_us", "std_dev_us",
              "p95_time_us", "p99_time_us", "load_imbalance_percent", "bandwidth_gbps"):
        assert _close(got[k], ref[k]), (k, got[k], ref[k])
    assert got["per_rank_means_us"] == pytest.approx(ref["per_rank_means_us"], rel=1e-9)
    assert got["mpi_implementation"] == ref["mpi_implementation"]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(F3, "results", "*.json"))))
def test_3d_stats_match_reference(path):
    ref = json.load(open(os.path.join(F3, "stats", os.path.basename(path)[:-5] + "_stats.json")))
    got = stats3d.stats_for_result(json.load(open(path)))
    for k in ("mean_time_ms", "median_time_ms", "min_time_ms", "max_time_ms", "tensor_size_mb"):
        assert _close(got[k], ref[k]), (k, got[k], ref[k])
    for k in ("implementation", "operation", "num_ranks", "hidden_dim", "seq_len", "batch"):
        assert got[k] == ref[k]


def test_1d_csv_layout_and_headline_row(tmp_path):
    rows = stats1d.process_directory(os.path.join(F1, "results"), str(tmp_path), verbose=False)
    assert rows
    with open(tmp_path / "benchmark_statistics.csv") as f:
        header = next(csv.reader(f))
    assert header == stats1d.LEGACY_COLUMNS
    # reference collectives/1d/stats/dsccl/benchmark_statistics.csv:22 (the 7.53 GB/s headline)
    r = [x for x in rows if x["mpi_implementation"] == "deepspeed_oneccl"
         and x["num_ranks"] == 2 and x["data_size_name"] == "16MB"][0]
    assert _close(r["median_time_us"], 1114.3472511321306)
    assert _close(r["bandwidth_gbps"], 13.274022312444641)
    # nccl-tests busBW at p50 on the true 8 MiB (7.53 GB/s)
    assert r["busbw_gbps"] == pytest.approx(7.53, abs=0.01)
    assert os.path.exists(tmp_path / "benchmark_statistics_ext.csv")
    assert os.path.exists(tmp_path / "benchmark_statistics_transpose.csv")


def test_3d_csv_layout(tmp_path):
    rows = stats3d.process_directory(os.path.join(F3, "results"), str(tmp_path), "ref",
                                     verbose=False)
    with open(tmp_path / "benchmark_statistics_3d_ref_standard.csv") as f:
        rd = list(csv.reader(f))
    assert rd[0] == stats3d.STANDARD_COLUMNS
    assert len(rd) == len(rows) + 1
    with open(tmp_path / "benchmark_statistics_3d_ref_transpose.csv") as f:
        tr = list(csv.reader(f))
    assert tr[0][0] == "Metric" and tr[0][1].startswith("allgather_r4_h4096_s1_b1")
    assert [r[0] for r in tr[1:5]] == ["mean_time_ms", "median_time_ms", "min_time_ms",
                                        "max_time_ms"]
    assert "--- Metadata ---" in [r[0] for r in tr if r]


def test_bandwidth_conventions():
    P, nb, t = 8, 1 << 20, 1e-3
    assert bus_factor("allreduce", P) == pytest.approx(2 * 7 / 8)
    assert busbw_gbps("allreduce", nb, t, P) == pytest.approx(nb / t / 1e9 * 1.75)
    assert algbw_gbps("allgather", nb, t, P) == pytest.approx(8 * nb / t / 1e9)
    assert busbw_gbps("allgather", nb, t, P) == pytest.approx(8 * nb / t / 1e9 * 7 / 8)
    assert busbw_gbps("reduce_scatter", nb, t, P) == pytest.approx(nb / t / 1e9 * 7 / 8)
    assert busbw_gbps("broadcast", nb, t, P) == pytest.approx(nb / t / 1e9)
    assert busbw_gbps("allreduce", nb, t, 1) == 0.0
    assert legacy_bandwidth_gbps(4194304, 1.0, 2) == pytest.approx(4194304 * 4 / 2 ** 30)


def test_compare_reference_against_itself_reproduces_baseline_numbers(tmp_path):
    """The comparison table's reference side reproduces BASELINE.md's busBW figures."""
    import glob

    from distributed_llm_backend_benchmark_amd.stats import compare as C

    fx = os.path.join(os.path.dirname(__file__), "fixtures", "reference")
    ref1 = C.load_1d(sorted(glob.glob(os.path.join(fx, "1d", "csv", "*.csv"))))
    rows = C.compare(ref1, ref1)
    assert rows and all(abs(r["speedup_p50"] - 1.0) < 1e-12 for r in rows)
    best = {(r["operation"], r["ref_num_ranks"], r["config"]): r for r in rows}
    r = best[("allreduce", 2, "16MB")]            # BASELINE: oneCCL P=2 8 MiB -> 7.53 GB/s
    assert r["ref_impl"] == "deepspeed_oneccl" and abs(r["ref_busbw_gbps"] - 7.53) < 0.01
    assert abs(best[("allreduce", 2, "1KB")]["ref_p50_us"] - 22.9) < 0.05   # OpenMPI best
    ref3 = C.load_3d(glob.glob(os.path.join(fx, "3d", "csv", "*.csv")))
    r3 = {(r["operation"], r["ref_num_ranks"], r["config"]): r for r in C.compare(ref3, ref3)}
    assert abs(r3[("allreduce", 8, "8/2048/2048")]["ref_busbw_gbps"] - 5.46) < 0.01
    C.write_csv(rows, str(tmp_path / "c.csv"))
    assert "| allreduce |" in C.markdown(rows)
