#!/bin/bash
# All-reduce algorithm / tuning variants on one node — the analogue of the reference's oneCCL
# sweep (collectives/3d/launch_dsccl.sh:34-65: CCL_ALLREDUCE algorithms, CCL_WORKER_COUNT,
# CCL_FUSION) and of its result dirs dsccl_<algo>_allreduce / dscclworker<k>.
#   usage: launch/allreduce_variants.sh [NGPUS]
set -uo pipefail
N=${1:-8}
export HSA_ENABLE_IPC_MODE_LEGACY=0
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29513}"
M="-m distributed_llm_backend_benchmark_amd.cli.collectives --mode 3d --ops allreduce --batch-sizes 8,16 --seq-lengths 2048,4096 --hidden-dims 2048,4096 --resume --validate"
run() { timeout -k 10 3600 $L $M "$@" || exit $?; }
run --impl-name rccl_default --output-dir results/3d/rccl_default
for algo in Ring Tree; do run --env NCCL_ALGO=$algo --impl-name rccl_${algo,,}_allreduce --output-dir results/3d/rccl_${algo,,}_allreduce; done
for proto in Simple LL128 LL; do run --env NCCL_PROTO=$proto --impl-name rccl_proto_${proto,,} --output-dir results/3d/rccl_proto_${proto,,}; done
for ch in 8 16 32 64; do run --env NCCL_MIN_NCHANNELS=$ch --env NCCL_MAX_NCHANNELS=$ch --impl-name rccl_channels$ch --output-dir results/3d/rccl_channels$ch; done
run --allreduce-impl custom --allreduce-algo twoshot --impl-name custom_twoshot_allreduce --output-dir results/3d/custom_twoshot_allreduce
# small/medium messages: one-shot IPC kernel vs RCCL (latency)
timeout -k 10 3600 $L -m distributed_llm_backend_benchmark_amd.cli.collectives --mode 1d --ops allreduce --sizes 512B:8MiB --dtype bf16 --allreduce-impl custom --allreduce-algo oneshot --impl-name custom_oneshot_allreduce --output-dir results/1d/custom_oneshot_allreduce --resume --validate --batched --graph
timeout -k 10 3600 $L -m distributed_llm_backend_benchmark_amd.cli.collectives --mode 1d --ops allreduce --sizes 512B:8MiB --dtype bf16 --impl-name rccl_small --output-dir results/1d/rccl_small --resume --validate --batched --graph
for d in results/3d/rccl_* results/3d/custom_*; do python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 3d --input-dir $d --output-dir stats/3d/$(basename $d) --impl $(basename $d); done
for d in results/1d/custom_oneshot_allreduce results/1d/rccl_small; do python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 1d --input-dir $d --output-dir stats/1d/$(basename $d); done
# one table per variant against the reference's oneCCL algorithm variants (dsccl_<algo>_allreduce)
REF=${REF_ROOT:-/root/reference}
if [ -d "$REF/collectives/3d/stats" ]; then
  for d in stats/3d/rccl_* stats/3d/custom_*; do
    python -m distributed_llm_backend_benchmark_amd.cli.compare --mode 3d --any-ranks --ours $d/benchmark_statistics_3d_$(basename $d)_ext.csv --ref $REF/collectives/3d/stats/*/benchmark_statistics_3d_*_standard.csv --output $d/compare_vs_reference.csv > $d/compare_vs_reference.md
  done
fi
