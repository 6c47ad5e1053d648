#!/bin/bash
# GPT-2 step (world 1) with the current kernels + the small-GEMM probe.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/step; mkdir -p $O
timeout -k 10 300 python tools/diag/gpt2_small_gemm_probe.py > $O/gpt2_small_gemm_probe.jsonl 2> $O/probe_err.log || { tail -20 $O/probe_err.log; exit 1; }
cat $O/gpt2_small_gemm_probe.jsonl
timeout -k 10 400 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 1; }
tail -2 $O/gpt2.log
DLBB_GEMM_PERSIST_EPI=0 timeout -k 10 400 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2_nopersist_epi.json > $O/gpt2_nopersist.log 2>&1 || { tail -20 $O/gpt2_nopersist.log; exit 1; }
tail -2 $O/gpt2_nopersist.log
