#!/bin/bash
# PMC counter runs (kernel-trace + stats + pmc only; no sys/runtime traces).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export PYTHONPATH=$R TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
P3="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
P4="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for t in "$@"; do
  for p in ${PASSES:-1 2}; do
    eval "C=\$P$p"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc $C --output-format csv \
      -d "$R/gpurun_out/pmc_${t}_p$p" -o pmc -- python3 "$R/tools/prof_target.py" "$t" \
      > "$R/gpurun_out/pmc_${t}_p$p.log" 2>&1
    rc=$?; echo "pmc $t pass $p rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_${t}_p$p.log"; exit $rc; fi
  done
done
