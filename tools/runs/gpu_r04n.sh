#!/bin/bash
# Round 4: why the GPT-2 loss trajectory moved (10.41 -> 10.32 at step 35): LM-head kernel
# numerics and the step under three settings on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/r04n
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  tail -3 "$R/$O/$name.log" | cut -c1-300
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step lmhead 200 python -u tools/diag/loss_ab.py
T="python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
step a_default 200 $T --output $O/a_default.json
step b_margin0 200 env DLBB_LIB_MARGIN=0 $T --output $O/b_margin0.json
step c_margin0_conc 200 env DLBB_LIB_MARGIN=0 DLBB_ATTN_CONCURRENT=1 $T --output $O/c_margin0_conc.json
step d_lmhead_mfma_conc 200 env DLBB_ATTN_CONCURRENT=1 $T --output $O/d_conc.json
for f in a_default b_margin0 c_margin0_conc d_conc; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['loss'], d['ms_per_step'])"; done
