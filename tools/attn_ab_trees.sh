#!/bin/bash
# Attention A/B of two source trees on one box: ./ab_old (a `git archive` of the base commit with
# its own in-tree build) against the working tree, interleaved rounds of the forward and backward
# timers (tools/attn_fwd_ab_trees.py, tools/attn_bwd_ab_trees.py; each prints one JSON line with
# the times and an output digest). Usage on the box: bash tools/attn_ab_trees.sh OUTFILE ROUNDS
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
N=${2:-3}
mkdir -p "$(dirname "$OUT")"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
: > "$OUT"
for i in $(seq 1 "$N"); do
  for t in old new; do
    if [ "$t" = old ]; then T=$R/ab_old; else T=$R; fi
    for k in fwd bwd; do
      line=$(cd "$T" && PYTHONPATH=$T timeout -k 10 120 python "$R/tools/attn_${k}_ab_trees.py") \
        || { echo "$k $t $i failed"; exit 1; }
      echo "{\"round\": $i, \"tree\": \"$t\", \"kernel\": \"$k\", \"r\": $line}" >> "$OUT"
      echo "$t $k $i: $(echo "$line" | cut -c1-300)"
    done
  done
done
