#!/bin/bash
# Ad-hoc GPU step runner for iteration: build, then each argument is a command run under its own
# time limit (600 s), stopping at the first failure / fault. Logs in gpurun_out/q<i>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
i=0
for c in "$@"; do
  i=$((i+1))
  echo "=== q$i: $c"
  timeout -k 10 600 bash -c "$c" > gpurun_out/q$i.log 2>&1
  rc=$?
  tail -4 gpurun_out/q$i.log
  echo "=== q$i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
