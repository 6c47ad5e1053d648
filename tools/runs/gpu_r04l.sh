#!/bin/bash
# Round 4: bench.py with 8 ranks sharing ONE GPU over a gloo process group (DLBB_BENCH_BACKEND=
# gloo): the P = 8 code path of the headline, sweep and the BASELINE config 3 / 4 / 5 sections
# (reduced shapes; the times are meaningless, 8 processes on one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04l
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLBB_BENCH_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 5 --warmup 2 \
  --shape 2,512,1024 --sweep-max-mib 16 --grid "2,512,1024;1,1024,1024" --moe "512,1024" \
  --ddp-model 2,2,128,1024,2,64 --ddp-steps 3 --config-budget-s 120 > $O/bench8.log 2>&1
rc=$?; tail -c 3000 $O/bench8.log; exit $rc
