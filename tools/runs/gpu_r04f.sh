#!/bin/bash
# Round 4 evidence: smoke, bench (world 1), TP 7B forward (graph replay default / eager), shards
# at P = 2/4/8, the overlapped shard-4 forward with a 300 GB/s link stand-in, the GPT-2 DDP step,
# and rocprofv3 kernel stats of the TP 7B forward and the GPT-2 step. First failing step ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/r04f
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  tail -2 "$R/$O/$name.log"
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
TP="python -m distributed_llm_backend_benchmark_amd.cli.run_tp --config config/7b_config.yaml --backend rccl"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step tp7b 300 $TP --output-dir $O/tp
step tp7b_eager 300 $TP --eager --output-dir $O/tp_eager
for P in 2 4 8; do
  step tp7b_shard$P 300 $TP --shard-as $P --output-dir $O/tp_shard$P
done
step tp7b_shard4_ov 300 $TP --shard-as 4 --emulate-busbw 300 --overlap-chunks 2 --output-dir $O/tp_shard4_ov
step gpt2 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json
step gpt2_emu100 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --emulate-comm 100 --comm-timeline --output $O/gpt2_emu100.json
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
step prof_tp7b 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_tp7b" -o tp7b -- python3 -m distributed_llm_backend_benchmark_amd.cli.run_tp --config "$R/config/7b_config.yaml" --backend rccl --output-dir "$R/$O/tp_prof"
step prof_gpt2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_gpt2" -o gpt2 -- python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
step pp_phases 200 python3 "$R/tools/diag/pp_phases.py" --nj 4 --shapes 4096x4096x4096,4096x4096x16384
echo done
