"""Interleaved in-process A/B of the GPT-2 DDP step (world 1) over named settings.

Each run builds a fresh trainer (cli/train_ddp.run) with the settings applied; the variants
alternate round by round on one box, so box-to-box spread does not enter the comparison.
One JSON line per run.

  base           the tree's defaults
  no_presort     embedding backward sorts the token ids itself (ops/embedding.PRESORT)
  col_one_pass   LayerNorm dgamma/dbeta column reduce in one 48-workgroup pass
  old            no_presort + col_one_pass (the round-6 start)
  split_cap=N    weight-gradient split-K capped at N (ops/gemm.set_wgrad_split_cap)

    python tools/step_ab.py --variants base,old,no_presort,col_one_pass --reps 3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def apply(name):
    import importlib

    from distributed_llm_backend_benchmark_amd.ops import _lib, gemm

    # (the package re-exports the embedding FUNCTION under the module's name)
    embedding = importlib.import_module("distributed_llm_backend_benchmark_amd.ops.embedding")

    embedding.PRESORT[0] = True
    _lib.lib().dlbb_layernorm_set_col_two_pass(1)
    gemm.set_wgrad_split_cap(None)
    if name in ("no_presort", "old"):
        embedding.PRESORT[0] = False
    if name in ("col_one_pass", "old"):
        _lib.lib().dlbb_layernorm_set_col_two_pass(0)
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
