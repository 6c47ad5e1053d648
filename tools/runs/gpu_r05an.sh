#!/bin/bash
# Round 5 pass an: confirmation on the final tree — DDP / stream tests, bench.py (driver
# contract), four GPT-2 step runs with their stream re-check records
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05an
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_comm_gpu.py tests/test_streams_gpu.py tests/test_attention_gpu.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python -u bench.py
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in 1 2 3 4; do
  step gpt2_$rep 300 $T --output $O/gpt2_$rep.json
  python -c "import json; d=json.load(open('$O/gpt2_$rep.json')); print('RESULT $rep', round(d['ms_per_step'],3), d['side_stream_checks'])"
done
