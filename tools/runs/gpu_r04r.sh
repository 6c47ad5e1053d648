#!/bin/bash
# Round 4: triple-buffered dK/dV slice ring — numerics, device times, GPT-2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/${RUN_TAG:-r04r}
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  tail -3 "$R/$O/$name.log" | cut -c1-400
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py -m gpu
step attn_bench 240 python -u tools/attn_bench.py
step gpt2 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json
echo done
