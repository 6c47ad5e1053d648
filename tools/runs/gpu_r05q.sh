#!/bin/bash
# Round 5 pass q: AdamW of each head bucket issued during backward (DLBB_OPT_OVERLAP=1 own
# stream, 2 on the weight-gradient side stream) vs the head range after backward (0): bit-exact
# test, then the GPT-2 step A/B interleaved, then a kernel trace of mode 1 for the timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05q
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_comm_gpu.py \
  -k "overlapped_optimizer or gpt2_training_step_hip_graph or emulated_comm or gpt2_ddp_step_world1"
step wgradpp 300 python -u tools/bench_kernels.py wgradpp
grep "^{" $O/wgradpp.log | cut -c1-600
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b c; do
  for ov in 0 1 2; do
    step gpt2_ov${ov}_$rep 300 env DLBB_OPT_OVERLAP=$ov $T --output $O/gpt2_ov${ov}_$rep.json
    python -c "import json; d=json.load(open('$O/gpt2_ov${ov}_$rep.json')); print('RESULT ov$ov $rep', round(d['ms_per_step'],3))"
  done
done
cd /tmp
export DLBB_OPT_OVERLAP=1
step prof_ov1 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_ov1" -o t -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
f=$(find $O/prof_ov1 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/stream_timeline.py "$f" --steps 3 > $O/timeline_ov1.jsonl
gzip -c "$f" > $O/trace_ov1.csv.gz; rm -f "$f"
cut -c1-300 $O/timeline_ov1.jsonl
