#!/bin/bash
# Round 5 pass f: GPT-2 step, eager vs whole-step HIP graph replay, and the
# graph under the HIP runtime's graph-execution knobs (packet capture off, parallel graph queues
# forced to 1 / 2 / 4); then kernel traces of eager and graph replay for the per-stream timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05f
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
for run in eager graph graph_nopc graph_q1 graph_q2 graph_q4 eager2 graph2; do
  case $run in
    eager*) step gpt2_$run 300 $T --output $O/gpt2_$run.json ;;
    graph|graph2) step gpt2_$run 300 $T --graph --output $O/gpt2_$run.json ;;
    graph_nopc) step gpt2_$run 300 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $T --graph --output $O/gpt2_$run.json ;;
    graph_q*) step gpt2_$run 300 env DEBUG_HIP_FORCE_GRAPH_QUEUES=${run#graph_q} $T --graph --output $O/gpt2_$run.json ;;
  esac
  python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
done
cd /tmp
for mode in eager graph; do
  extra=""; [ $mode = graph ] && extra="--graph"
  step prof_$mode 600 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$mode" -o t -- \
    python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3 $extra
  f=$(find $O/prof_$mode -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/stream_timeline.py "$f" --steps 3 > $O/timeline_$mode.jsonl
  gzip -c "$f" > $O/trace_$mode.csv.gz; rm -f "$f"
  cut -c1-400 $O/timeline_$mode.jsonl
done
