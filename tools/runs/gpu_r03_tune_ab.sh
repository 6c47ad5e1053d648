#!/bin/bash
# A/B on one box, GPT-2 step world 1: autotune timing (single-call medians vs interleaved
# best-of-reps) x sink weight gradients on a side stream (off / on), two interleaved rounds.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tune_ab; mkdir -p $O
for r in 1 2; do
  for tt in single interleaved; do
    for ws in 0 1; do
      n=${tt}_ws${ws}_r$r
      DLBB_TUNE_TIMING=$tt DLBB_WGRAD_STREAM=$ws timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/$n.json > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
      echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(round(d['ms_per_step'],3), d['gemm_kernel_mix']['hand_written_time_fraction'])")"
    done
  done
done
