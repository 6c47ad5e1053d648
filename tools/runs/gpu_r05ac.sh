#!/bin/bash
# Round 5 pass ac: cap the weight-gradient workgroups per CU by padding their LDS request
# (DLBB_WGRAD_MIN_LDS_KB), so the compute stream's LN / attention kernels keep room on every CU;
# GPT-2 step A/B interleaved (workgroup budget scaled to the slots left)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05ac
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 env DLBB_WGRAD_MIN_LDS_KB=64 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad_matches or wgrad_wide or wgrad_256"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  for cfg in "base:" "l54:DLBB_WGRAD_MIN_LDS_KB=54" "l54s:DLBB_WGRAD_MIN_LDS_KB=54 DLBB_WGRAD_SLOTS=0.667" "l80:DLBB_WGRAD_MIN_LDS_KB=80 DLBB_WGRAD_SLOTS=0.667"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    step gpt2_${name}_$rep 300 env $envs $T --output $O/gpt2_${name}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_${name}_$rep.json')); print('RESULT $name $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
