#!/bin/bash
# Round 4: what bounds the GPT-2 LM-head forward — tile order (GROUP_M) sweep, then PMC passes
# (MFMA busy / waits, L2 hit / miss / HBM requests, UTCL1 translation hit / miss) for our 256²
# persistent kernel, the 256 x 192 spread-store kernel and hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/r04h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u tools/diag/lmhead_order.py > $O/order.jsonl 2> $O/order.err
rc=$?; echo "order rc=$rc"; cat $O/order.jsonl; [ $rc -ne 0 ] && exit $rc
PASSES="1 2 3" bash tools/gpu_pmc.sh lmhead lmhead192p lmheadblas
