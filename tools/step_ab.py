"""Interleaved in-process A/B of the GPT-2 DDP step (world 1) over named settings.

Each run builds a fresh trainer (cli/train_ddp.run) with the settings applied; the variants
alternate round by round on one box, so box-to-box spread does not enter the comparison.
One JSON line per run.

  base           the tree's defaults
  split_cap=N    weight-gradient split-K capped at N (ops/gemm.set_wgrad_split_cap)
  wgrad_fused    weight-gradient split-K combined in-launch (ops/gemm.set_wgrad_fused)
  no_wgrad_side  weight gradients on the compute stream (parallel/ddp._WGRAD_STREAM)

(Round 6 also ran a two-pass LayerNorm column reduce and the embedding token sort moved into the
forward on a side stream through this tool — profiles/r06_step/step_ab_presort_colreduce.jsonl,
commit bc963df — both slower in the step, removed.)

    python tools/step_ab.py --variants base,split_cap=4 --reps 3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_DEFAULT_WGRAD_STREAM = [None]


def apply(name):
    from distributed_llm_backend_benchmark_amd.ops import gemm
    from distributed_llm_backend_benchmark_amd.parallel import ddp

    gemm.set_wgrad_split_cap(None)
    gemm.set_wgrad_fused(False)
    ddp._WGRAD_STREAM = _DEFAULT_WGRAD_STREAM[0]
    if name == "wgrad_fused":
        gemm.set_wgrad_fused(True)
    if name == "no_wgrad_side":
        ddp._WGRAD_STREAM = False
    if name.startswith("split_cap="):
        gemm.set_wgrad_split_cap(int(name.split("=")[1]))
        gemm.WGRAD_CHOICES.clear()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base,old")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()

    from distributed_llm_backend_benchmark_amd.cli import train_ddp
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    from distributed_llm_backend_benchmark_amd.parallel import ddp

    _DEFAULT_WGRAD_STREAM[0] = ddp._WGRAD_STREAM
    comm = init_distributed("auto")
    args = train_ddp.parse_args(["--steps", str(a.steps), "--warmup", str(a.warmup)])
    for rep in range(a.reps):
        for name in a.variants.split(","):
            apply(name)
            res = train_ddp.run(args, comm, overlap=True)
            print(json.dumps({"rep": rep, "variant": name, "ms_per_step": res["ms_per_step"],
                              "side_stream_checks": res["side_stream_checks"]}), flush=True)
    apply("base")
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
