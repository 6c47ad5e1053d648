#!/bin/bash
# Round 5 pass ad: loss normaliser / mean as two one-workgroup kernels (were seven torch
# launches) and the unit-upstream mark (no scaling passes in the LM-head backward): tests, then
# the GPT-2 step with the mark on / off, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05ad
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_comm_gpu.py -k "xent or unit_upstream or gpt2 or cross_entropy or loss"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  for u in 1 0; do
    step gpt2_u${u}_$rep 300 env DLBB_UNIT_UPSTREAM=$u $T --output $O/gpt2_u${u}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_u${u}_$rep.json')); print('RESULT u$u $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
