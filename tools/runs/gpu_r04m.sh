#!/bin/bash
# Round 4: delta fused into the dQ kernel, LayerNorm backward fallback widths — numerics,
# attention device times, the GPT-2 step, then bench.py with 8 ranks sharing ONE GPU over gloo
# (the P = 8 path of the headline, sweep and BASELINE config 3 / 4 / 5 sections, reduced shapes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/${RUN_TAG:-r04m}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  tail -3 "$R/$O/$name.log" | cut -c1-300
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_kernels_gpu.py -k "attn or attention or layernorm" -m gpu
step attn_bench 240 python -u tools/attn_bench.py
step gpt2 300 python -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 30 --warmup 5 --output $O/gpt2.json
step bench8 900 env DLBB_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 5 --warmup 2 \
  --shape 2,512,1024 --sweep-max-mib 16 --grid "2,512,1024;1,1024,1024" --moe "512,1024" \
  --ddp-model 2,2,128,1024,2,64 --ddp-steps 3 --config-budget-s 120
echo done
