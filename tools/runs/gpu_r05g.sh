#!/bin/bash
# Round 5 pass g: split-K reduce variants (isolated + in the GPT-2 step), LN-backward variant in
# the step, then pass f (graph vs eager) and pass e (8-rank IPC probe) — the probe last.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05g
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step kb 300 python -u tools/bench_kernels.py splitred
cat $O/kb.log | grep split_reduce | cut -c1-400
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b; do
  for cfg in "0 0" "2 0" "1 0" "2 1"; do
    set -- $cfg
    run=sr$1_ln$2_$rep
    step gpt2_$run 300 env DLBB_SPLIT_REDUCE_VARIANT=$1 DLBB_LN_BWD_VARIANT=$2 $T --output $O/gpt2_$run.json
    python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
  done
done
bash tools/runs/gpu_r05f.sh && bash tools/runs/gpu_r05e.sh
