#!/bin/bash
# Round 4: PMC passes of the attention kernels at the GPT-2 shape (what bounds them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PASSES="1 4" bash tools/gpu_pmc.sh attnfwd attnbwd
