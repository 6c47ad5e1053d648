#!/bin/bash
# Round 5 pass v: attention backward incremental DMA sources (tests + interleaved A/B), then the
# GPT-2 step with the new attention defaults vs the old ones (forward variant 0, backward 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05v
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py
step ab 300 python -u tools/diag/attn_bwd_incr.py
grep "^{" $O/ab.log | cut -c1-400
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b; do
  step gpt2_old_$rep 300 env DLBB_ATTN_FWD_VARIANT=0 DLBB_ATTN_BWD_INCR=0 $T --output $O/gpt2_old_$rep.json
  python -c "import json; d=json.load(open('$O/gpt2_old_$rep.json')); print('RESULT old $rep', round(d['ms_per_step'],3))"
  step gpt2_new_$rep 300 $T --output $O/gpt2_new_$rep.json
  python -c "import json; d=json.load(open('$O/gpt2_new_$rep.json')); print('RESULT new $rep', round(d['ms_per_step'],3))"
  step gpt2_new3_$rep 300 env DLBB_ATTN_BWD_INCR=3 $T --output $O/gpt2_new3_$rep.json
  python -c "import json; d=json.load(open('$O/gpt2_new3_$rep.json')); print('RESULT new3 $rep', round(d['ms_per_step'],3))"
done
