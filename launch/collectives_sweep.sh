#!/bin/bash
# 1D + 3D collective sweeps at 1/2/4/8 GPUs (replaces collectives/launch_{openmpi,intelmpi,dsccl}.sh).
#   usage: launch/collectives_sweep.sh "1 2 4 8" [results_root]
# Writes results/<mode>/rccl/*.json (+ stats/) per rank count; --resume makes it restartable.
set -uo pipefail
COUNTS=${1:-"1 2 4 8"}; ROOT=${2:-results}
export HSA_ENABLE_IPC_MODE_LEGACY=0
M=distributed_llm_backend_benchmark_amd.cli.collectives
for n in $COUNTS; do
  L="python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29512}"
  timeout -k 10 3600 $L -m $M --mode 1d --dtype bf16 --sizes 1KiB:1GiB --ops allreduce,allgather,reduce_scatter,broadcast,reduce,alltoall,sendrecv --batched --graph --resume --output-dir $ROOT/1d/rccl || exit $?
  timeout -k 10 3600 $L -m $M --mode 1d --dtype bf16 --sizes 1KiB:1GiB --ops allreduce,allgather,reduce_scatter,broadcast,reduce,alltoall,sendrecv --engine native --impl-name rccl_native --batched --graph --resume --output-dir $ROOT/1d/rccl_native || exit $?
  timeout -k 10 3600 $L -m $M --mode 1d --dtype fp16 --sizes reference --resume --output-dir $ROOT/1d/rccl_reference || exit $?
  timeout -k 10 3600 $L -m $M --mode 3d --resume --output-dir $ROOT/3d/rccl || exit $?
  timeout -k 10 3600 $L -m $M --mode 3d --ops alltoall_moe --batch-sizes 1 --seq-lengths 4096,16384 --hidden-dims 4096,7168 --resume --output-dir $ROOT/3d/rccl_moe || exit $?
done
python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 1d --input-dir $ROOT/1d/rccl --output-dir stats/1d/rccl
python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 1d --input-dir $ROOT/1d/rccl_native --output-dir stats/1d/rccl_native
python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 1d --input-dir $ROOT/1d/rccl_reference --output-dir stats/1d/rccl_reference
python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 3d --input-dir $ROOT/3d/rccl --output-dir stats/3d/rccl --impl rccl
