#!/bin/bash
# Round 5 pass aa: side-stream forks without the system-scope fence of a default HIP event
# (DLBB_FORK_EVENT nofence / device / torch): DDP + graph tests, GPT-2 step A/B interleaved, and a
# kernel trace of the default to check the compute stream's gaps after forked-from kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05aa
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_comm_gpu.py -k "gpt2 or ddp or overlapped or cu_share or tied"
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  for m in torch nofence device; do
    step gpt2_${m}_$rep 300 env DLBB_FORK_EVENT=$m $T --output $O/gpt2_${m}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_${m}_$rep.json')); print('RESULT $m $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
step gpt2_graph 300 $T --graph --output $O/gpt2_graph.json
python -c "import json; d=json.load(open('$O/gpt2_graph.json')); print('RESULT graph', round(d['ms_per_step'],3), d['loss'])"
cd /tmp
step prof 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o t -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
gzip -c "$f" > $O/trace_nofence.csv.gz; rm -f "$f"
