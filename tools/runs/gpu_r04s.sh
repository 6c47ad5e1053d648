#!/bin/bash
# Round 4: PMC passes of the single-round long-K NT GEMM (4096 x 4096 x 16384), ours vs hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PASSES="1 2 4" bash tools/gpu_pmc.sh longk longkblas
