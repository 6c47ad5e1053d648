#!/bin/bash
# Round 5 pass ab: kernel traces of the GPT-2 step per fork-event mode (the nofence trace showed
# ~100 us compute-stream gaps after forked-from kernels under rocprofv3 only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05ab
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cd /tmp
for m in torch device nofence; do
  echo "=== prof $m $(date +%T)"
  DLBB_FORK_EVENT=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$m" -o t -- \
    python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3 --output $O/gpt2_prof_$m.json > $O/prof_$m.log 2>&1; rc=$?
  echo "=== prof $m rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  f=$(find $O/prof_$m -name "*kernel_trace.csv" | head -1)
  gzip -c "$f" > $O/trace_$m.csv.gz; rm -f "$f"
done
