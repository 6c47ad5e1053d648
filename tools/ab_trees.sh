#!/bin/bash
# A/B of two source trees on one box: ./ab_old (a `git archive` of the previous commit with its
# own in-tree build) against the working tree, interleaved. Usage on the box:
#   bash tools/ab_trees.sh OUTDIR ROUNDS
# Per round: tools/wgrad_shapes_bench.py under each tree, then one GPT-2 DDP world-1 run per tree
# (separate processes, each tree's package first on sys.path).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/$1
N=${2:-3}
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for i in $(seq 1 "$N"); do
  for t in old new; do
    if [ "$t" = old ]; then T=$R/ab_old; else T=$R; fi
    (cd "$T" && PYTHONPATH=$T timeout -k 10 120 python "$R/tools/wgrad_shapes_bench.py" \
      > "$O/wg_${t}_$i.json" 2> "$O/wg_${t}_$i.err") || { echo "wg $t $i failed"; exit 1; }
    (cd "$T" && PYTHONPATH=$T timeout -k 10 120 python -m \
      distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 20 --warmup 5 \
      --output "$O/step_${t}_$i.json" > "$O/step_${t}_$i.log" 2>&1) || { echo "step $t $i failed"; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/step_${t}_$i.json')); print('$t', $i, round(d['ms_per_step'], 3))"
  done
done
