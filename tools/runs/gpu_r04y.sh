#!/bin/bash
# Round 4: GPT-2 step eager vs whole-step HIP graph replay (world 1), same box, back to back.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04y
mkdir -p $O
T="python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for run in eager graph eager2 graph2; do
  extra=""; case $run in graph*) extra="--graph";; esac
  timeout -k 10 200 $T $extra --output $O/$run.json > $O/$run.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('$O/$run.json')); print('$run', round(d['ms_per_step'],3), d['hip_graph'], d['loss'])"
done
