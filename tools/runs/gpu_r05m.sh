#!/bin/bash
# Round 5 pass m: memcpy / memset nodes in a replayed graph (branch concurrency), and the
# collective-path memory kernels under rocprofv3 --stats (kernel names for the roofline table).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05m
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step gb 180 python -u tools/diag/graph_branches.py
cd /tmp
step prof_mem 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_mem" -o mem -- python3 $R/tools/bench_kernels.py memroof
cd "$R"
f=$(find $O/prof_mem -name "*kernel_trace.csv" | head -1); rm -f "$f"
ls $O/prof_mem
bash tools/runs/gpu_r05n.sh
