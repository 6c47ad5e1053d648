#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 300 python -u tools/diag/lmhead_grad_ab.py > $O/grad_ab.log 2>&1
rc=$?; tail -8 $O/grad_ab.log; exit $rc
