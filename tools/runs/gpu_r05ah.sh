#!/bin/bash
# Round 5 pass ah: AdamW of the tied table's untouched rows right after the LM-head backward
# (DLBB_EARLY_ROWS): bit-exact tests + DDP/graph tests, then the GPT-2 step on / off interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05ah
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_comm_gpu.py -k "early_rows or gpt2 or ddp or overlapped or tied or zero2 or unit_upstream"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  for e in 1 0; do
    step gpt2_e${e}_$rep 300 env DLBB_EARLY_ROWS=$e $T --output $O/gpt2_e${e}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_e${e}_$rep.json')); print('RESULT e$e $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
step gpt2_graph 300 $T --graph --output $O/gpt2_graph.json
python -c "import json; d=json.load(open('$O/gpt2_graph.json')); print('RESULT graph', round(d['ms_per_step'],3), d['loss'])"
