#!/bin/bash
# PMC passes over one tools/prof_target.py target, one rocprofv3 run per counter group (counters +
# kernel trace only), summarised by tools/pmc_summary.py. Usage on the box:
#   bash tools/pmc_target.sh TARGET OUTDIR MATCH "C1 C2 ..." ["C5 C6 ..." ...]
set -eu
T=$1; O=$GRAFT_REPO_ROOT/$2; M=$3; shift 3
mkdir -p "$O"
export PYTHONPATH=$GRAFT_REPO_ROOT HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for grp in "$@"; do
  i=$((i + 1))
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp \
    --output-format csv -d "$O/p$i" -o t -- python3 "$GRAFT_REPO_ROOT/tools/prof_target.py" "$T")
done
cd "$GRAFT_REPO_ROOT"
for j in $(seq 1 $i); do python3 tools/pmc_summary.py "$O/p$j" --match "$M"; done \
  > "$O/summary.jsonl"
rm -rf "$O"/p*
cat "$O/summary.jsonl"
