#!/bin/bash
# Round 5 pass ap: stream-pairing flips with 4 vs 8 hardware queues per process (8 runs each)
# hipBLASLt runs at step time? 8 runs default vs 8 with the library never chosen
# (DLBB_LIB_MARGIN=10), interleaved; each run records its warm-up stream re-checks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05ap
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
T="python -u -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 10 --warmup 4"
for rep in 1 2 3 4 5 6 7 8; do
  for m in q4 q8; do
    envs="GPU_MAX_HW_QUEUES=4"; [ $m = q8 ] && envs="GPU_MAX_HW_QUEUES=8"
    timeout -k 10 200 env $envs $T --output $O/gpt2_${m}_$rep.json > $O/gpt2_${m}_$rep.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('$O/gpt2_${m}_$rep.json')); print('RESULT $m $rep', round(d['ms_per_step'],3), [c['serialised'] for c in d['side_stream_checks']], d['gemm_kernel_mix']['linear']['tuned'][-1]['choice'])"
  done
done
