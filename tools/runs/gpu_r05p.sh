#!/bin/bash
# Round 5 pass p: NT ping-pong with wave row 0's B(u+2) LDS-DMA pieces spread one per 16 MFMAs
# inside its MFMA phase (set_stagger(12)) vs the balanced default (7) and the clumped form (11),
# on the TP-7B shapes at P = 1 / 2 and the GPT-2 LM head, against hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05p
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "moveb or moveab"
step table 600 python -u tools/tp_gemm_table.py --ps 1,2 --modes s7,s12,s13 --lmhead
cat $O/table.log | grep '^{' | cut -c1-400
step table2 600 python -u tools/tp_gemm_table.py --ps 1,2 --modes s13,s12,s7 --lmhead
