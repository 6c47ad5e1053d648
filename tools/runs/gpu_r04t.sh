#!/bin/bash
# Round 4: ping-pong with row 0's B DMA inside its MFMA phase (mode 11) — numerics, then the 7B /
# GPT-2 GEMM table against mode 7 (BAL) and hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/${RUN_TAG:-r04t}
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
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_plain or gemm_epi" -m gpu
step table 400 python -u tools/tp_gemm_table.py --ps 1,2,4,8 --gpt2 --modes s7,s11 --rounds 5
echo done
