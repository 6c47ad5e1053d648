"""bench.py's BASELINE config 3/4/5 sections on the CPU (gloo, world 2, tiny shapes): every
section present and validated, and a section that fails (injected) is recorded as an error
without changing the headline record."""

import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SMALL = ["--shape", "1,64,256", "--sweep-max-mib", "1", "--grid", "1,64,256;2,32,256",
         "--moe", "64,256", "--ddp-model", "2,2,64,256,2,32", "--ddp-steps", "2"]
HEADLINE_KEYS = ("metric", "unit", "n_gpus", "steps", "warmup", "higher_is_better", "scaling",
                 "dtype", "config")


def _bench(extra_env=None):
    from launch_utils import run_torchrun

    env = {k: v for k, v in os.environ.items() if k != "CUDA_VISIBLE_DEVICES"}
    env.update(extra_env or {})
    out = run_torchrun(2, [os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3",
                           "--warmup", "1"] + SMALL, 300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def _check_sections(cfgs):
    c3 = cfgs["config3_3d_allgather_reduce_scatter"]
    assert [r["shape"] for r in c3["rows"]] == [[1, 64, 256], [2, 32, 256]]
    for row in c3["rows"]:
        for op in ("allgather", "reduce_scatter"):
            assert row[op]["best"] == "rccl" and row[op]["busbw_GBps"] > 0, row
    c4 = cfgs["config4_moe_alltoall"]
    assert c4["rows"][0]["best"] == "rccl" and c4["rows"][0]["busbw_GBps"] > 0
    c5 = cfgs["config5_gpt2_ddp"]
    assert c5["best"] == "rccl" and c5["global_batch"] == 4 and c5["tokens_per_s"] > 0
    assert c5["by_allreduce"]["rccl"]["bucket_paths"] == {"rccl": c5["by_allreduce"]["rccl"]
                                                          ["buckets"]}


def test_bench_sections_and_isolated_failure():
    ok = _bench()
    _check_sections(ok["baseline_configs"])
    bad = _bench({"DLBB_BENCH_FAIL_SECTION": "config3:1"})
    cfgs = bad["baseline_configs"]
    err = cfgs["config3_3d_allgather_reduce_scatter"]["error"]
    # rank 1 failed alone; the agreement made every rank leave the section together
    assert "injected failure" in err and "rank(s) [1]" in err, err
    # the other sections still ran, and the headline record has the same shape and fields
    assert cfgs["config4_moe_alltoall"]["rows"] and cfgs["config5_gpt2_ddp"]["best"] == "rccl"
    for k in HEADLINE_KEYS:
        assert bad[k] == ok[k], k
    assert bad["value"] > 0 and bad["vs_baseline"] is not None


def test_section_wrapper_world1_error_record():
    """run_section at world 1: a raising section returns {"error"} and seconds, never raises."""
    from distributed_llm_backend_benchmark_amd.bench.baseline_configs import run_section
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo")
    try:
        def boom(c, b):
            raise ValueError("nope")

        rec = run_section(comm, "x", boom, 10)
        assert rec["error"] == "ValueError: nope" and rec["failed_ranks"] == [0]
        rec = run_section(comm, "y", lambda c, b: {"v": 1, "left": b.seconds}, 10)
        assert rec["v"] == 1 and rec["left"] == 10 and rec["seconds"] >= 0
    finally:
        comm.destroy()
