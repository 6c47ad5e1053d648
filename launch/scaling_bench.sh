#!/bin/bash
# bench.py at 1, 2, 4, 8 GPUs back to back (what the driver does for SCALE_rNN.json).
set -uo pipefail
for n in ${1:-1 2 4 8}; do
  if [ "$n" = 1 ]; then timeout -k 10 600 python bench.py --gpus 1 || exit $?
  else timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n || exit $?; fi
done
