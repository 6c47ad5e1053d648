#!/bin/bash
# Round 5 pass o: graph replay vs eager under more hardware queues per process (the graph
# runtime's internal branch streams may share the launch stream's queue when the process already
# holds many streams); the kernel sort vs torch.sort in the step (DLBB_SORT_IDS=torch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05o
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b; do
  for q in 4 8 16; do
    step gpt2_eager_q${q}_$rep 300 env GPU_MAX_HW_QUEUES=$q $T --output $O/gpt2_eager_q${q}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_eager_q${q}_$rep.json')); print('RESULT eager q$q $rep', round(d['ms_per_step'],3))"
    step gpt2_graph_q${q}_$rep 300 env GPU_MAX_HW_QUEUES=$q $T --graph --output $O/gpt2_graph_q${q}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_graph_q${q}_$rep.json')); print('RESULT graph q$q $rep', round(d['ms_per_step'],3))"
  done
  step gpt2_torchsort_$rep 300 env DLBB_SORT_IDS=torch $T --output $O/gpt2_torchsort_$rep.json
  python -c "import json; d=json.load(open('$O/gpt2_torchsort_$rep.json')); print('RESULT torchsort $rep', round(d['ms_per_step'],3))"
done
cd /tmp
step prof_graph16 300 env GPU_MAX_HW_QUEUES=16 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_graph16" -o t -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3 --graph
f=$(find $O/prof_graph16 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/stream_timeline.py "$f" --steps 3 > $O/timeline_graph16.jsonl
gzip -c "$f" > $O/trace_graph16.csv.gz; rm -f "$f"
cut -c1-300 $O/timeline_graph16.jsonl
