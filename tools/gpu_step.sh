#!/bin/bash
# One gpurun call = a list of steps, each under its own time limit, stopping at the first
# failure (a hang, fault or abort ends the call). Usage on the box:
#   bash tools/gpu_step.sh OUTDIR "name1|timeout1|cmd1" "name2|timeout2|cmd2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; shift
mkdir -p "$O"
export PYTHONPATH=$(pwd) HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" bash -c "$cmd" > "$O/$name.log" 2>&1; rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
