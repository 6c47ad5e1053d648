#!/bin/bash
# rocprofv3 kernel-trace + stats of the flagship paths (no PMC counters here; counters get a
# separate run). Outputs land in gpurun_out/prof_*/ ; summaries are copied to profiles/ by hand.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export PYTHONPATH=$R TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"; timeout -k 10 "$t" "$@" > "$R/gpurun_out/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$R/gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
}
for what in "$@"; do case $what in
  tp) step prof_tp 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_tp" -o tp -- \
        python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config "$R/config/7b_config.yaml" \
        --backend rccl --warmup 1 --iters 3 --output-dir "$R/gpurun_out/tp" ;;
  gpt2) step prof_gpt2 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_gpt2" -o gpt2 -- \
        python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 5 --warmup 2 ;;
  bench) step prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench" -o bench -- \
        python3 "$R/bench.py" --steps 20 --warmup 5 ;;
  kbench) step kbench 900 python3 "$R/tools/bench_kernels.py" gemm mem ;;
  tpbench) step tp7b 900 python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config "$R/config/7b_config.yaml" --backend rccl --output-dir "$R/gpurun_out/tp" &&
           step tp7b_torch 900 python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config "$R/config/7b_config.yaml" --backend rccl --kernels torch --output-dir "$R/gpurun_out/tp_torch" ;;
  gpt2bench) step gpt2 900 python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 20 --warmup 5 --output "$R/gpurun_out/gpt2.json" &&
           step gpt2_torch 900 env DLBB_KERNELS=torch python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 20 --warmup 5 --output "$R/gpurun_out/gpt2_torch.json" ;;
  sweep1) M=distributed_llm_backend_benchmark_amd.cli.collectives
        step sweep1d 900 python3 -m $M --mode 1d --dtype bf16 --sizes 1KiB:1GiB --ops allreduce,allgather,reduce_scatter,broadcast,reduce,alltoall,sendrecv --batched --graph --validate --iters 50 --output-dir "$R/gpurun_out/results/r01_world1/1d/rccl" &&
        step sweep1d_ref 900 python3 -m $M --mode 1d --dtype fp16 --sizes reference --validate --output-dir "$R/gpurun_out/results/r01_world1/1d/rccl_reference" &&
        step sweep3d 900 python3 -m $M --mode 3d --batch-sizes 1,8,32 --seq-lengths 1,2048,8192 --hidden-dims 2048,4096 --iters 30 --validate --output-dir "$R/gpurun_out/results/r01_world1/3d/rccl" &&
        step stats1d 300 python3 -m distributed_llm_backend_benchmark_amd.cli.stats --mode 1d --input-dir "$R/gpurun_out/results/r01_world1/1d/rccl" --output-dir "$R/gpurun_out/results/r01_world1/stats/1d/rccl" &&
        step stats3d 300 python3 -m distributed_llm_backend_benchmark_amd.cli.stats --mode 3d --input-dir "$R/gpurun_out/results/r01_world1/3d/rccl" --output-dir "$R/gpurun_out/results/r01_world1/stats/3d/rccl" --impl rccl ;;
  census) step census 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_census" -o census -- \
        python3 -m pytest "$R/tests" -m gpu -q -p no:cacheprovider -x ;;
esac; done
