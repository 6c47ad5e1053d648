#!/bin/bash
# Round 5 pass d (first pass of the resumed session): kernel tests of the round-5 paths, memory /
# LN-backward / wgrad-combine microbenchmarks, GPT-2 step LN-backward A/B, steady-state rocprof
# table of the step, and the default bench.py run (driver contract) with its wall time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05d
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "wgrad or layernorm or cast or chunk" \
  tests/test_comm_gpu.py::test_allgather_list_form_unpack_bit_exact_world1
step kb 600 python -u tools/bench_kernels.py lnab wgradfused wgradsplit memroof
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 20 --warmup 5"
for run in ln1 ln0 ln1b ln0b; do
  case $run in
    ln1*) step gpt2_$run 300 $T --output $O/gpt2_$run.json ;;
    ln0*) step gpt2_$run 300 env DLBB_LN_BWD_VARIANT=0 $T --output $O/gpt2_$run.json ;;
  esac
  python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('RESULT $run', round(d['ms_per_step'],3), d['loss'])"
done
cd /tmp
step prof_gpt2 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_gpt2" -o gpt2 -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
cd "$R"
f=$(find $O/prof_gpt2 -name "*kernel_trace.csv" | head -1)
python tools/prof_steady.py "$f" --marker adamw_kernel --skip 6 --csv $O/gpt2_kernel_stats_steady.csv > $O/steady.txt
head -30 $O/steady.txt | cut -c1-200
rm -f "$f"
