#!/bin/bash
# Round 5 pass c: GPT-2 step A/B of stream arrangements (main stream high priority, weight
# gradients serial) and eager vs whole-step HIP graph replay; kernel traces of eager and graph
# replay for the per-stream timeline (tools/stream_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05c
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for run in base hp serial graph base2 hp2 serial2 graph2; do
  case $run in
    base*) step gpt2_$run 300 $T --output $O/gpt2_$run.json ;;
    hp*) step gpt2_$run 300 $T --main-stream-priority -1 --output $O/gpt2_$run.json ;;
    serial*) step gpt2_$run 300 env DLBB_WGRAD_STREAM=0 $T --output $O/gpt2_$run.json ;;
    graph*) step gpt2_$run 300 $T --graph --output $O/gpt2_$run.json ;;
  esac
  python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
done
cd /tmp
for mode in eager graph; do
  extra=""; [ $mode = graph ] && extra="--graph"
  step prof_$mode 600 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$mode" -o t -- \
    python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3 $extra
  f=$(find $O/prof_$mode -name "*kernel_trace.csv" | head -1)
  cp "$f" $O/trace_$mode.csv
  python3 $R/tools/stream_timeline.py $O/trace_$mode.csv --steps 3 > $O/timeline_$mode.jsonl
  cut -c1-400 $O/timeline_$mode.jsonl
done
