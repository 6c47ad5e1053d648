#!/bin/bash
# Round validation + evidence: full GPU test suite, smoke, bench (world 1), TP 7B forward,
# GPT-2 DDP step, rocprofv3 kernel stats of the GPT-2 step. Each GPU step has its own limit;
# the first failing step ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/final/$name.log" 2>&1
  local rc=$?
  tail -3 "$R/gpurun_out/final/$name.log"
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread --deselect tests/test_native_host_asan.py::test_host_asan_with_device
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step tp7b 600 python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl --output-dir gpurun_out/final/tp
for P in 2 4 8; do
  step tp7b_shard$P 300 python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl --shard-as $P --output-dir gpurun_out/final/tp_shard$P
done
step gpt2 600 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output gpurun_out/final/gpt2.json
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
step prof_tp7b 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/final/prof_tp7b" -o tp7b -- python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config "$R/config/7b_config.yaml" --backend rccl --output-dir "$R/gpurun_out/final/tp_prof"
step prof_gpt2 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/final/prof_gpt2" -o gpt2 -- python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 5 --warmup 2
[ -x build/asan/host_checks ] && step asan_probe 200 bash -c "cd $R && ASAN_OPTIONS=detect_leaks=1:verify_asan_link_order=0 LSAN_OPTIONS=suppressions=$R/tests/native/lsan.supp timeout -k 5 150 build/asan/host_checks" || echo "asan probe skipped (build/asan is gpurun-ignored; run tools/build_host_asan.py and un-ignore to include it)"
echo done
