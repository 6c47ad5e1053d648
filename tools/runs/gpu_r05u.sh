#!/bin/bash
# Round 5 pass u: attention forward schedule variants — numerics tests, interleaved A/B, PMC of
# the default and the fastest variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05u
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py
step ab 300 python -u tools/diag/attn_fwd_variants.py
grep "^{" $O/ab.log | cut -c1-700
cd /tmp
for v in 0 7; do
  echo "=== pmc v$v $(date +%T)"
  DLBB_ATTN_FWD_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d "$O/pmc_v$v" -o p -- python3 $R/tools/diag/attn_pmc.py > $O/pmc_v$v.log 2>&1; rc=$?
  echo "=== pmc v$v rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, json, sys, collections
O = sys.argv[1]
for v in (0, 7):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{O}/pmc_v{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "attn_fwd" not in r["Kernel_Name"]:
                continue
            agg["fwd"][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {c: round(sum(x) / len(x)) for c, x in agg["fwd"].items()}
    print("PMC v%d" % v, json.dumps(out))
PY
