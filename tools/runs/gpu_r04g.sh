#!/bin/bash
# Round 4: persistent 256 x 192 NT GEMM with spread C stores (variant 2) — numerics, then the
# GPT-2 forward GEMM table (LM head and the plain-output shapes) against the 256 x 192 ping-pong
# and hipBLASLt, then the GPT-2 step with the new candidate in the autotuner.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/${RUN_TAG:-r04g}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  tail -3 "$R/$O/$name.log"
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step numerics 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "spread or tile_variants" -m gpu
step table 300 python -u tools/tp_gemm_table.py --ps 1,2,4 --gpt2 --modes auto,v192,v192p,v192p18 --rounds 5
step gpt2 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json
echo done
