#!/bin/bash
# Round 5 pass e: 8-ranks-on-one-GPU direct IPC probe — full matrix with
# per-call host timings per rank, at 4 ranks (default queues), 8 ranks (default = 4 HW queues
# per process) and 8 ranks with 2 HW queues per process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05e
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for cfg in "4 default" "8 default" "8 2"; do
  set -- $cfg
  d=$O/w$1_q$2
  echo "=== world $1 queues $2 $(date +%T)"
  timeout -k 10 230 python -u tools/diag/ipc8_probe.py $d $1 $2 > $d.log 2>&1; rc=$?
  echo "=== rc=$rc"; tail -3 $d.log | cut -c1-300
  for f in $d/rank*.jsonl; do echo "$f $(wc -l < $f) $(tail -1 $f | cut -c1-200)"; done
  if [ $rc -ne 0 ]; then exit $rc; fi
done
