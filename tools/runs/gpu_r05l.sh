#!/bin/bash
# Round 5 pass l: weight gradients dealt over k side streams (eager and graph), the graph probe
# with round-robin side streams, the n-way reduce forms (tests + memory roofline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05l
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
  tests/test_kernels_gpu.py tests/test_comm_gpu.py -k "reduce or ddp or graph or capture"
step gb 180 python -u tools/diag/graph_branches.py
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b; do
  for k in 1 2 3; do
    step gpt2_k${k}_$rep 300 env DLBB_WGRAD_STREAMS=$k $T --output $O/gpt2_k${k}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_k${k}_$rep.json')); print('RESULT k$k $rep', round(d['ms_per_step'],3), d['loss'])"
    step gpt2_graph_k${k}_$rep 300 env DLBB_WGRAD_STREAMS=$k $T --graph --output $O/gpt2_graph_k${k}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_graph_k${k}_$rep.json')); print('RESULT graph k$k $rep', round(d['ms_per_step'],3), d['loss'])"
  done
done
step kb 600 python -u tools/bench_kernels.py memroof
grep reduce_sum $O/kb.log | cut -c1-300
