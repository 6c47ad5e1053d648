#!/bin/bash
# Round 5 pass w: GPT-2 step with the weight gradients on the unsplit 256^2 TN ping-pong
# (DLBB_WGRAD_IMPL=pp: 2.2x fewer CU-microseconds per dW than the split-K 128 x 256 tiles, but
# ~330 us latency per call on 9-36 CUs) dealt over 1 / 2 / 4 side streams, vs the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05w
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad_forced_pp or wgrad_matches or pingpong_tn"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b; do
  for cfg in "base:" "pp1:DLBB_WGRAD_IMPL=pp DLBB_WGRAD_STREAMS=1" "pp2:DLBB_WGRAD_IMPL=pp DLBB_WGRAD_STREAMS=2" "pp4:DLBB_WGRAD_IMPL=pp DLBB_WGRAD_STREAMS=4" "base4:DLBB_WGRAD_STREAMS=4"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    step gpt2_${name}_$rep 300 env $envs $T --output $O/gpt2_${name}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_${name}_$rep.json')); print('RESULT $name $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
