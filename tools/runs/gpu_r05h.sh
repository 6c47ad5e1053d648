#!/bin/bash
# Round 5 pass h: asm transposed LDS reads (no compiler vmcnt(0) drain of the LDS-DMA prefetch)
# in the NN / TN ping-pong GEMMs, the weight-gradient kernel and the attention kernels:
# correctness (kernel tests), kernel tables vs hipBLASLt / torch, the GPT-2 step with A/Bs
# (split-K reduce variant, LN-backward variant), steady-state rocprof table; then pass f
# (graph vs eager) and pass e (8-rank IPC probe) last.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05h
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_attention_gpu.py
step attn 300 python -u tools/attn_bench.py
step gemm_gpt2 600 python -u tools/gpt2_gemm_table.py
step kb 300 python -u tools/bench_kernels.py splitred wgradsplit lnab
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5"
for rep in a b; do
  for cfg in "2 0" "0 0" "2 1"; do
    set -- $cfg
    run=sr$1_ln$2_$rep
    step gpt2_$run 300 env DLBB_SPLIT_REDUCE_VARIANT=$1 DLBB_LN_BWD_VARIANT=$2 $T --output $O/gpt2_$run.json
    python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
  done
done
cd /tmp
step prof_gpt2 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_gpt2" -o gpt2 -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
cd "$R"
f=$(find $O/prof_gpt2 -name "*kernel_trace.csv" | head -1)
python tools/prof_steady.py "$f" --marker adamw_kernel --skip 6 --csv $O/gpt2_kernel_stats_steady.csv > $O/steady.txt
head -24 $O/steady.txt | cut -c1-160
python3 tools/stream_timeline.py "$f" --steps 3 > $O/timeline_eager.jsonl || true
rm -f "$f"
bash tools/runs/gpu_r05f.sh && bash tools/runs/gpu_r05e.sh
