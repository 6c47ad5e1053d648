#!/bin/bash
# Code-path rehearsal of the driver's 8-rank bench.py on ONE GPU: 8 ranks share the card over a
# gloo process group (DLBB_BENCH_BACKEND=gloo; times meaningless, never reported as numbers).
# A heartbeat line every 50 s keeps the silent phases (gloo all-reduces of 64 MiB among 8 ranks
# on one card) visible. Usage on the box: bash tools/rehearse_bench8.sh OUT.json
set -u
OUT=$1
(while true; do sleep 50; echo "heartbeat $(date +%T)"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
DLBB_BENCH_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --standalone \
  --local-addr 127.0.0.1 --nproc-per-node 8 bench.py --gpus 8 --steps 5 --warmup 2 \
  --deadline-s 420 > "$OUT.log" 2>&1
rc=$?
grep '^{' "$OUT.log" | tail -1 > "$OUT"
echo "rehearsal rc=$rc"
exit $rc
