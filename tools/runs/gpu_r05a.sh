#!/bin/bash
# Round 5 first GPU pass: kernel tests of the new paths, A/B microbenchmarks (LN backward,
# in-launch wgrad split-K combine, memory kernels), GPT-2 step A/B, steady-state rocprof table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/r05a
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -4 "$O/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "wgrad or layernorm or cast or chunk" tests/test_comm_gpu.py::test_allgather_list_form_unpack_bit_exact_world1
step kb 600 python -u tools/bench_kernels.py lnab wgradfused memroof
cp $O/kb.log $O/kb.jsonl
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 20 --warmup 5"
for run in new old new2 old2; do
  case $run in
    new*) step gpt2_$run 300 $T --output $O/gpt2_$run.json ;;
    old*) step gpt2_$run 300 env DLBB_WGRAD_FUSED=0 DLBB_LN_BWD_VARIANT=0 $T --output $O/gpt2_$run.json ;;
  esac
  python -c "import json; d=json.load(open('$O/gpt2_$run.json')); print('$run', round(d['ms_per_step'],3), d['loss'])"
done
cd /tmp
step prof_gpt2 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_gpt2" -o gpt2 -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 8 --warmup 3
cd "$R"
f=$(find $O/prof_gpt2 -name "*kernel_trace.csv" | head -1)
python tools/prof_steady.py "$f" --marker adamw_kernel --skip 6 --csv $O/gpt2_kernel_stats_steady.csv | head -30
