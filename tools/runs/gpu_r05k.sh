#!/bin/bash
# Round 5 pass k: why the captured GPT-2 step loses its side-stream overlap under graph replay —
# branch probe with mid-graph forks (the DDP backward's pattern), the captured step's topology
# (hipGraphDebugDotPrint via DLBB_GRAPH_DOT) — plus the weight-gradient workgroup budget above 1
# and the attention tests on the reverted forward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05k
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_attention_gpu.py tests/test_kernels_gpu.py -k "attn or split"
step gb 120 python -u tools/diag/graph_branches.py
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
step gpt2_graph_dot 300 env DLBB_GRAPH_DOT=$O/gpt2_step.dot $T --graph --output $O/gpt2_graph_dot.json
python tools/diag/graph_dot.py $O/gpt2_step.dot | tee $O/gpt2_step_topology.json | cut -c1-400
gzip -f $O/gpt2_step.dot
for rep in a b; do
  for sl in 1.0 1.5 2.0; do
    run=slots${sl}_$rep
    step gpt2_$run 300 env DLBB_WGRAD_SLOTS=$sl $T --output $O/gpt2_$run.json
    python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
  done
done
