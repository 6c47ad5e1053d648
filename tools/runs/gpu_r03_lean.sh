#!/bin/bash
# Lean persistent epilogues: GPU numerics tests, then the GPT-2 small-GEMM probe (A/B).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/probe; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${TESTK:-persistent_lean or gemm_epilogues or gemm_plain or dgrad}" > $O/pytest_lean.log 2>&1 || { tail -30 $O/pytest_lean.log; exit 1; }
tail -2 $O/pytest_lean.log
timeout -k 10 300 python tools/diag/gpt2_small_gemm_probe.py > $O/gpt2_small_gemm_probe_lean.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
cat $O/gpt2_small_gemm_probe_lean.jsonl
