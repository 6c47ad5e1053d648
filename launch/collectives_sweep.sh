#!/bin/bash
# 1D + 3D collective sweeps at 1/2/4/8 GPUs (replaces collectives/launch_{openmpi,intelmpi,dsccl}.sh),
# then stats and the like-for-like comparison with the reference's published CSVs.
#   usage: launch/collectives_sweep.sh "1 2 4 8" [results_root] [stats_root]
# Every config is validated against its closed form (--validate) and refused if its timing is
# below the memory / xGMI roofline (bench/sweep.py roofline_guard); --resume makes it restartable.
set -uo pipefail
COUNTS=${1:-"1 2 4 8"}; ROOT=${2:-results}; STATS=${3:-stats}
export HSA_ENABLE_IPC_MODE_LEGACY=0
M=distributed_llm_backend_benchmark_amd.cli.collectives
REF=${REF_ROOT:-/root/reference}
for n in $COUNTS; do
  L="python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29512}"
  V="--validate --resume"
  timeout -k 10 3600 $L -m $M --mode 1d --dtype bf16 --sizes 1KiB:1GiB --ops allreduce,allgather,reduce_scatter,broadcast,reduce,alltoall,sendrecv --batched --graph $V --output-dir $ROOT/1d/rccl || exit $?
  timeout -k 10 3600 $L -m $M --mode 1d --dtype bf16 --sizes 1KiB:1GiB --ops allreduce,allgather,reduce_scatter,broadcast,reduce,alltoall,sendrecv --engine native --impl-name rccl_native --batched --graph $V --output-dir $ROOT/1d/rccl_native || exit $?
  timeout -k 10 3600 $L -m $M --mode 1d --dtype fp16 --sizes reference $V --output-dir $ROOT/1d/rccl_reference || exit $?
  timeout -k 10 3600 $L -m $M --mode 3d $V --output-dir $ROOT/3d/rccl || exit $?
  if [ "$n" -gt 1 ]; then
    timeout -k 10 3600 $L -m $M --mode 3d --ops allgather,reduce_scatter,alltoall --direct-ipc --impl-name rccl_direct $V --output-dir $ROOT/3d/rccl_direct || exit $?
  fi
  timeout -k 10 3600 $L -m $M --mode 3d --ops alltoall_moe --batch-sizes 1 --seq-lengths 4096,16384 --hidden-dims 4096,7168 $V --output-dir $ROOT/3d/rccl_moe || exit $?
done
S="python -m distributed_llm_backend_benchmark_amd.cli.stats"
$S --mode 1d --input-dir $ROOT/1d/rccl --output-dir $STATS/1d/rccl
$S --mode 1d --input-dir $ROOT/1d/rccl_native --output-dir $STATS/1d/rccl_native
$S --mode 1d --input-dir $ROOT/1d/rccl_reference --output-dir $STATS/1d/rccl_reference
$S --mode 3d --input-dir $ROOT/3d/rccl --output-dir $STATS/3d/rccl --impl rccl
[ -d $ROOT/3d/rccl_direct ] && $S --mode 3d --input-dir $ROOT/3d/rccl_direct --output-dir $STATS/3d/rccl_direct --impl rccl_direct
$S --mode 3d --input-dir $ROOT/3d/rccl_moe --output-dir $STATS/3d/rccl_moe --impl rccl_moe
# like-for-like tables against the reference's published CSVs
C="python -m distributed_llm_backend_benchmark_amd.cli.compare"
if [ -d "$REF/collectives" ]; then
  $C --mode 1d --ours $STATS/1d/rccl_reference/benchmark_statistics_ext.csv --ref $REF/collectives/1d/stats/*/benchmark_statistics.csv --output $STATS/compare_1d_vs_reference.csv > $STATS/compare_1d_vs_reference.md
  $C --mode 3d --ours $STATS/3d/rccl/benchmark_statistics_3d_rccl_ext.csv --ref $REF/collectives/3d/stats/*/benchmark_statistics_3d_*_standard.csv --output $STATS/compare_3d_vs_reference.csv > $STATS/compare_3d_vs_reference.md
else
  F=tests/fixtures/reference
  $C --mode 1d --ours $STATS/1d/rccl_reference/benchmark_statistics_ext.csv --ref $F/1d/csv/*.csv --output $STATS/compare_1d_vs_reference.csv > $STATS/compare_1d_vs_reference.md
  $C --mode 3d --ours $STATS/3d/rccl/benchmark_statistics_3d_rccl_ext.csv --ref $F/3d/csv/*.csv --output $STATS/compare_3d_vs_reference.csv > $STATS/compare_3d_vs_reference.md
fi
