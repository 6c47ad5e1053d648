#!/bin/bash
# Round 5 pass ae: stream priorities — weight-gradient side stream low (1) and/or the compute
# stream high (-1), GPT-2 step interleaved x3 (the slow-run pattern: compute-stream kernels
# waiting for CU space the side stream's weight-gradient workgroups took first)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05ae
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step prange 120 python -c "import torch; print('priority range', torch.cuda.Stream(priority=5).priority, torch.cuda.Stream(priority=-5).priority)"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  for cfg in "base:" "wlow:DLBB_WGRAD_STREAM_PRIORITY=1" "mhigh:" "both:DLBB_WGRAD_STREAM_PRIORITY=1"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    extra=""
    case $name in mhigh|both) extra="--main-stream-priority -1" ;; esac
    step gpt2_${name}_$rep 300 env $envs $T $extra --output $O/gpt2_${name}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_${name}_$rep.json')); print('RESULT $name $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
