#!/bin/bash
# Round 5 pass ar: AdamW with non-temporal fp32 state traffic (DLBB_ADAMW_NT): bit-exact test,
# GPT-2 step on / off interleaved x3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05ar
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adamw"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  for nt in 1 0; do
    step gpt2_nt${nt}_$rep 300 env DLBB_ADAMW_NT=$nt $T --output $O/gpt2_nt${nt}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_nt${nt}_$rep.json')); print('RESULT nt$nt $rep', round(d['ms_per_step'],3), d['loss'], [c['serialised'] for c in d['side_stream_checks']])"
  done
done
