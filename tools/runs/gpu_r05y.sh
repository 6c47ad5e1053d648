#!/bin/bash
# Round 5 pass y: weight-gradient side stream confined to a CU share (hardware CU mask) —
# test, then the GPT-2 step A/B over shares and workgroup budgets, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05y
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_comm_gpu.py -k cu_share
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b; do
  for cfg in "base:" "s14:DLBB_WGRAD_CU_SHARE=1/4 DLBB_WGRAD_SLOTS=0.25" "s38:DLBB_WGRAD_CU_SHARE=3/8 DLBB_WGRAD_SLOTS=0.375" "s12:DLBB_WGRAD_CU_SHARE=1/2 DLBB_WGRAD_SLOTS=0.5" "s12w:DLBB_WGRAD_CU_SHARE=1/2 DLBB_WGRAD_SLOTS=1.0" "s34:DLBB_WGRAD_CU_SHARE=3/4 DLBB_WGRAD_SLOTS=0.75"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    step gpt2_${name}_$rep 300 env $envs $T --output $O/gpt2_${name}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_${name}_$rep.json')); print('RESULT $name $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
