#!/bin/bash
# Round 5 pass t: PMC anatomy of the attention kernels at the GPT-2 shape (one counter set per
# rocprofv3 run, kernel-trace only besides --pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r05t
mkdir -p $O
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i + 1))
  echo "=== pmc$i $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$O/pmc$i" -o p -- \
    python3 $R/tools/diag/attn_pmc.py > $O/pmc$i.log 2>&1; rc=$?
  echo "=== pmc$i rc=$rc"; tail -2 $O/pmc$i.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, json, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{O}/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "attn" not in name:
            continue
        key = name.split("(")[0].replace("dlbb::", "")
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
json.dump(out, open(f"{O}/attn_pmc.json", "w"), indent=1)
for k, cs in out.items():
    print(k, {c: round(v) for c, v in sorted(cs.items())})
PY
