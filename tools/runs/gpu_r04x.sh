#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 400 python -u tools/diag/wgrad_split_sweep.py > $O/sweep.jsonl 2> $O/sweep.err
rc=$?; tail -3 $O/sweep.jsonl; exit $rc
