#!/bin/bash
# A/B: sink weight-gradient GEMMs on a probed side stream (DLBB_WGRAD_STREAM=1) vs inline, GPT-2
# step world 1, interleaved twice on one box.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wgrad_stream; mkdir -p $O
for r in 1 2; do
  for ws in 0 1; do
    DLBB_WGRAD_STREAM=$ws timeout -k 10 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2_ws${ws}_r$r.json > $O/gpt2_ws${ws}_r$r.log 2>&1 || { tail -20 $O/gpt2_ws${ws}_r$r.log; exit 1; }
    echo "ws=$ws r=$r $(python -c "import json;d=json.load(open('$O/gpt2_ws${ws}_r$r.json'));print(round(d['ms_per_step'],3))")"
  done
done
