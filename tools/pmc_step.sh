#!/bin/bash
# One rocprofv3 PMC pass over a short GPT-2 DDP world-1 run (counters only + kernel trace, no
# runtime traces): per kernel, waves resident per SIMD (SQ_WAVE_CYCLES vs kernel cycles) and MFMA
# busy — finds launch-shape / occupancy problems like the causal attention grid's.
# Usage on the box: bash tools/pmc_step.sh OUTDIR
set -eu
O=$GRAFT_REPO_ROOT/$1
mkdir -p "$O"
export PYTHONPATH=$GRAFT_REPO_ROOT HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/raw" -o step -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 3 --warmup 2
cd "$GRAFT_REPO_ROOT"
python3 tools/pmc_summary.py "$O/raw" > "$O/pmc_step_summary.jsonl"
rm -rf "$O/raw"
