#!/bin/bash
# Round 4: LM-head forward with and without its C stores (tile-order sweep + no-store diagnostic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${RUN_TAG:-r04i}
mkdir -p $O
timeout -k 10 240 python -u tools/diag/lmhead_order.py > $O/order.jsonl 2> $O/order.err
rc=$?; echo "order rc=$rc"; cat $O/order.jsonl; exit $rc
