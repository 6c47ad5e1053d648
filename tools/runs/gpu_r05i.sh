#!/bin/bash
# Round 5 pass i: 8-rank IPC tests at default queues with the gloo-leg calibration skipped;
# HIP-graph branch concurrency (tools/diag/graph_branches.py) under the runtime's graph knobs;
# GPT-2 eager vs graph without the side stream; main-stream priority; wgrad ring depth; the
# default bench.py run (driver contract).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05i
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests_k 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "split or wgrad or cast or chunk"
step tests_comm 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_comm_gpu.py -k "direct_ipc or calibration"
for kn in default q1 q2 q4 nopc; do
  case $kn in
    default) step gb_$kn 120 python -u tools/diag/graph_branches.py ;;
    nopc) step gb_$kn 120 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python -u tools/diag/graph_branches.py ;;
    q*) step gb_$kn 120 env DEBUG_HIP_FORCE_GRAPH_QUEUES=${kn#q} python -u tools/diag/graph_branches.py ;;
  esac
done
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for run in eager serial serial_graph hp eager2 serial2 serial_graph2 hp2; do
  case $run in
    eager*) step gpt2_$run 300 $T --output $O/gpt2_$run.json ;;
    serial_graph*) step gpt2_$run 300 env DLBB_WGRAD_STREAM=0 $T --graph --output $O/gpt2_$run.json ;;
    serial*) step gpt2_$run 300 env DLBB_WGRAD_STREAM=0 $T --output $O/gpt2_$run.json ;;
    hp*) step gpt2_$run 300 $T --main-stream-priority -1 --output $O/gpt2_$run.json ;;
  esac
  python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
done
step kb 300 python -u tools/bench_kernels.py wgradstages splitred
s=$(date +%s)
step bench 900 python -u bench.py
echo "bench wall $(( $(date +%s) - s )) s"
tail -1 $O/bench.log | cut -c1-600
# attention: software-pipelined operand reads (ab/attn_pipe: forward V^T groups, dQ K^T pairs)
# vs the tree's kernels, interleaved, and the variant's kernel tests
step attn_base 300 python -u tools/attn_bench.py
(cd ab/attn_pipe && PYTHONPATH=$R/ab/attn_pipe timeout -k 10 300 python -u tools/attn_bench.py > $O/attn_pipe.log 2>&1) && echo "attn_pipe ok"
step attn_base2 300 python -u tools/attn_bench.py
(cd ab/attn_pipe && PYTHONPATH=$R/ab/attn_pipe timeout -k 10 300 python -u tools/attn_bench.py > $O/attn_pipe2.log 2>&1) && echo "attn_pipe2 ok"
(cd ab/attn_pipe && PYTHONPATH=$R/ab/attn_pipe timeout -k 10 300 python -u -m pytest -x -q --timeout 120 -p no:cacheprovider tests/test_attention_gpu.py > $O/attn_pipe_tests.log 2>&1); echo "attn_pipe tests rc=$?"
# weight-gradient workgroup budget on the side stream (DLBB_WGRAD_SLOTS scale), GPT-2 step
for rep in a b; do
  for sl in 1.0 0.5 0.33; do
    run=slots${sl}_$rep
    step gpt2_$run 300 env DLBB_WGRAD_SLOTS=$sl $T --output $O/gpt2_$run.json
    python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
  done
done
