#!/bin/bash
# CPU plumbing run (BASELINE config 1): 1D fp32 all-reduce 1KB-1MB over Gloo, world 2.
set -euo pipefail
N=${1:-2}; OUT=${2:-results/1d/gloo}
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29511}" \
  -m distributed_llm_backend_benchmark_amd.cli.collectives --mode 1d --backend gloo \
  --dtype fp32 --ops allreduce --sizes 1KiB:1MiB --output-dir "$OUT" --impl-name gloo --validate
