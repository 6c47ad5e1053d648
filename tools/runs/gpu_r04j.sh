#!/bin/bash
# Round 4: attention backward with pre-negated / pre-scaled row constants and an unmasked
# interior path — numerics, then device times (tools/attn_bench.py) and the GPT-2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/${RUN_TAG:-r04j}
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  tail -4 "$R/$O/$name.log"
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step attn_tests 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py -m gpu
step attn_bench 240 python -u tools/attn_bench.py
step gpt2 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json

# (RUN_PROF=1) steady-state kernel table of the GPT-2 step
if [ "${RUN_PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
  step prof_gpt2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_gpt2" -o gpt2 -- python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
  cd "$R"
  step steady 60 python tools/prof_steady.py $O/prof_gpt2/gpt2_kernel_trace.csv --marker adamw_kernel --skip 6 --csv $O/gpt2_kernel_stats_steady.csv
fi
echo done-prof
