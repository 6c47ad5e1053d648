"""The reference's core deliverable end to end — 1D / 3D collective sweep, stats, comparison
with the reference's published CSVs (``collectives/1d/openmpi.py:204-300``,
``collectives/3d/dsccl.py:120-241``, ``collectives/1d/stats.py:135-288``) — as one helper shared
by the CPU (gloo), ranks-on-one-GPU (gloo over GPU tensors) and one-process-per-GPU (RCCL)
tests, so the multi-GPU test is the same code the rehearsals already run."""

import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(REPO, "tests", "fixtures", "reference")

OPS_1D = ["allreduce", "allgather", "reduce_scatter", "broadcast", "reduce", "gather", "scatter",
          "alltoall", "sendrecv"]
SIZES_1D = ["1KB", "1MB"]                       # reference labels (fp16 elements)
OPS_3D = ["allreduce", "allgather", "reduce_scatter", "alltoall"]
SHAPES_3D = dict(batch="1,8", seq="2048", hidden="2048")


def _run(cmd, timeout, env=None):
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO,
                         env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **(env or {})))
    assert out.returncode == 0, (cmd, out.stdout[-2000:], out.stderr[-4000:])
    return out


def _torchrun(nproc, args, timeout):
    from launch_utils import run_torchrun

    out = run_torchrun(nproc, ["-m", "distributed_llm_backend_benchmark_amd.cli.collectives"]
                       + args, timeout)
    assert out.returncode == 0, (out.args, out.stdout[-2000:], out.stderr[-4000:])
    return out


def run_pipeline(tmp, nproc, backend="rccl", device="auto", direct_ipc=False,
                 ops_1d=OPS_1D, ops_3d=OPS_3D, timeout=900):
    """Sweep -> stats -> compare. Returns the paths and the compare outputs."""
    tmp = str(tmp)
    common = ["--backend", backend, "--device", device, "--validate", "--warmup", "2",
              "--iters", "10"]
    _torchrun(nproc, ["--mode", "1d", "--dtype", "fp16", "--sizes", ",".join(SIZES_1D),
                      "--ops", ",".join(ops_1d), "--output-dir", f"{tmp}/res/1d/ours"] + common,
              timeout)
    impls = [("ours", [])] + ([("ours_direct", ["--direct-ipc"])] if direct_ipc else [])
    for label, extra in impls:
        ops = ops_3d if not extra else [o for o in ops_3d if o != "allreduce"]
        _torchrun(nproc, ["--mode", "3d", "--ops", ",".join(ops), "--batch-sizes",
                          SHAPES_3D["batch"], "--seq-lengths", SHAPES_3D["seq"],
                          "--hidden-dims", SHAPES_3D["hidden"], "--impl-name", label,
                          "--output-dir", f"{tmp}/res/3d/{label}"] + extra + common, timeout)
    m = [sys.executable, "-m"]
    _run(m + ["distributed_llm_backend_benchmark_amd.cli.stats", "--mode", "1d", "--input-dir",
              f"{tmp}/res/1d/ours", "--output-dir", f"{tmp}/st/1d/ours"], 300)
    for label, _ in impls:
        _run(m + ["distributed_llm_backend_benchmark_amd.cli.stats", "--mode", "3d",
                  "--input-dir", f"{tmp}/res/3d/{label}", "--output-dir", f"{tmp}/st/3d/{label}",
                  "--impl", label], 300)
    cmp1 = _run(m + ["distributed_llm_backend_benchmark_amd.cli.compare", "--mode", "1d",
                     "--ours", f"{tmp}/st/1d/ours/benchmark_statistics_ext.csv", "--ref"]
                + sorted(glob.glob(f"{FIX}/1d/csv/*.csv")) + ["--any-ranks", "--output",
                                                              f"{tmp}/cmp_1d.csv"], 300)
    cmp3 = _run(m + ["distributed_llm_backend_benchmark_amd.cli.compare", "--mode", "3d",
                     "--ours", f"{tmp}/st/3d/ours/benchmark_statistics_3d_ours_ext.csv",
                     "--ref"] + sorted(glob.glob(f"{FIX}/3d/csv/*.csv"))
                + ["--any-ranks", "--output", f"{tmp}/cmp_3d.csv"], 300)
    return {"tmp": tmp, "impls": [l for l, _ in impls], "cmp1": cmp1.stdout,
            "cmp3": cmp3.stdout}


def check_pipeline(res, nproc, ops_1d=OPS_1D, ops_3d=OPS_3D, busbw_positive=True):
    """Every config written (no error records), validated, and every raw record became a stats
    row (none refused by the roofline guard); busBW > 0 at P > 1; the comparison tables joined
    our rows with the reference's."""
    import csv

    tmp = res["tmp"]
    errs = glob.glob(f"{tmp}/res/**/*.error.json", recursive=True)
    assert not errs, [json.load(open(e))["error"] for e in errs]
    raw1 = sorted(glob.glob(f"{tmp}/res/1d/ours/*.json"))
    assert len(raw1) == len(ops_1d) * len(SIZES_1D), raw1
    nshapes = len(SHAPES_3D["batch"].split(",")) * len(SHAPES_3D["hidden"].split(","))
    for label in res["impls"]:
        ops = ops_3d if label == "ours" else [o for o in ops_3d if o != "allreduce"]
        raw3 = sorted(glob.glob(f"{tmp}/res/3d/{label}/*.json"))
        assert len(raw3) == len(ops) * nshapes, raw3
        for f in raw3:
            d = json.load(open(f))
            assert d["validated"] is True and d["num_ranks"] == nproc, f
            if label != "ours":
                assert d["op_impl"] == "custom", f
        rows = list(csv.DictReader(open(
            f"{tmp}/st/3d/{label}/benchmark_statistics_3d_{label}_ext.csv")))
        assert len(rows) == len(raw3)                   # nothing refused by the guard
        if busbw_positive:
            assert all(float(r["busbw_gbps"]) > 0 for r in rows), rows
    for f in raw1:
        d = json.load(open(f))
        assert d["validated"] is True, f
    rows = list(csv.DictReader(open(f"{tmp}/st/1d/ours/benchmark_statistics_ext.csv")))
    assert len(rows) == len(raw1)
    if busbw_positive:
        assert all(float(r["busbw_gbps"]) > 0 for r in rows), rows
    joined1 = list(csv.DictReader(open(f"{tmp}/cmp_1d.csv")))
    joined3 = list(csv.DictReader(open(f"{tmp}/cmp_3d.csv")))
    assert joined1 and joined3, (res["cmp1"], res["cmp3"])
