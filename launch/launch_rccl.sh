#!/bin/bash
# TP transformer forward benchmark on N MI355X GPUs of one node (run_mpi.py parity).
# Replaces launch_openmpi.sh / launch_intelmpi.sh (mpirun -np 4 --bind-to core ...):
# one process per GPU, LOCAL_RANK -> HIP device; RCCL over xGMI.
#   usage: launch/launch_rccl.sh [NGPUS] [CONFIG] [extra run_tp args...]
set -euo pipefail
N=${1:-4}; CFG=${2:-config/baseline_config.yaml}; shift $(( $# > 2 ? 2 : $# )) || true
export HSA_ENABLE_IPC_MODE_LEGACY=0
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-8}
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29510}" \
  -m distributed_llm_backend_benchmark_amd.cli.run_tp --config "$CFG" --backend rccl "$@"
