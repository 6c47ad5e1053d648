#!/bin/bash
# Round 5 pass n: the step without the torch.sort memcpy — eager vs graph replay A/B, and the
# graph replay's per-stream timeline (does the side-stream overlap survive capture now?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05n
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "sort or embedding or reduce" tests/test_comm_gpu.py -k "ddp or graph or capture or sort or embedding or reduce"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  step gpt2_eager_$rep 300 $T --output $O/gpt2_eager_$rep.json
  python -c "import json; d=json.load(open('$O/gpt2_eager_$rep.json')); print('RESULT eager $rep', round(d['ms_per_step'],3), d['loss'])"
  step gpt2_graph_$rep 300 $T --graph --output $O/gpt2_graph_$rep.json
  python -c "import json; d=json.load(open('$O/gpt2_graph_$rep.json')); print('RESULT graph $rep', round(d['ms_per_step'],3), d['loss'])"
done
cd /tmp
for mode in eager graph; do
  extra=""; [ $mode = graph ] && extra="--graph"
  step prof_$mode 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$mode" -o t -- \
    python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3 $extra
  f=$(find $O/prof_$mode -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/stream_timeline.py "$f" --steps 3 > $O/timeline_$mode.jsonl
  python3 $R/tools/prof_steady.py "$f" --marker adamw_kernel --skip 6 --csv $O/steady_$mode.csv > $O/steady_$mode.txt
  gzip -c "$f" > $O/trace_$mode.csv.gz; rm -f "$f"
  cut -c1-300 $O/timeline_$mode.jsonl
done
