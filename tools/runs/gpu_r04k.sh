#!/bin/bash
# Round 4 final evidence on the current tree: the whole GPU suite, smoke, bench (world 1),
# GPT-2 DDP step (default library margin / fastest-wins A/B / 100 GB/s stand-in), TP 7B forward
# and shards, steady-state rocprof kernel tables. First failing step ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/${RUN_TAG:-r04k}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  tail -2 "$R/$O/$name.log" | cut -c1-400
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gpu_tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step gpt2 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json
step gpt2_margin0 300 env DLBB_LIB_MARGIN=0 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2_margin0.json
step gpt2_emu100 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --emulate-comm 100 --comm-timeline --output $O/gpt2_emu100.json
step tp7b 300 $TP --output-dir $O/tp
for P in 2 4 8; do
  step tp7b_shard$P 300 $TP --shard-as $P --output-dir $O/tp_shard$P
done
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
step prof_gpt2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_gpt2" -o gpt2 -- python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
step prof_tp7b 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_tp7b" -o tp7b -- python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config "$R/config/7b_config.yaml" --backend rccl --output-dir "$R/$O/tp_prof"
cd "$R"
step steady_gpt2 60 python tools/prof_steady.py $O/prof_gpt2/gpt2_kernel_trace.csv --marker adamw_kernel --skip 6 --csv $O/gpt2_kernel_stats_steady.csv
echo done
