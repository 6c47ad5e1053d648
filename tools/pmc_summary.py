"""Summarise rocprofv3 PMC counter CSVs: per kernel name, median over dispatches of each counter,
plus derived MFMA-busy %, wait %, L2 hit %, and DRAM bytes (EA RDREQ/WRREQ x 64 B; see the
MI355X guide for the FETCH_SIZE caveat)."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def load(d):
    rows = list(csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))))
    per = defaultdict(lambda: defaultdict(list))
    for r in rows:
        per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    byk = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, vs in cs.items():
            byk[k][c].append(sum(vs))
    dur = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "pmc_kernel_trace.csv"))):
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return byk, dur


def main(root, targets):
    out = []
    for t in targets:
        merged = defaultdict(dict)
        durs = {}
        for p in (1, 2):
            d = os.path.join(root, f"pmc_{t}_p{p}")
            if not os.path.isdir(d):
                continue
            byk, dur = load(d)
            for k, cs in byk.items():
                for c, vs in cs.items():
                    merged[k][c] = statistics.median(vs)
                durs[k] = statistics.median(dur.get(k, [0]))
        for k, cs in merged.items():
            if k.startswith("__amd") or "distribution" in k or "elementwise" in k:
                continue
            wc = cs.get("SQ_WAVE_CYCLES", 0)
            line = {"target": t, "kernel": k[:70], "dur_us": durs.get(k, 0) / 1e3}
            if wc:
                line["wait_any_%"] = 100 * cs["SQ_WAIT_ANY"] / wc
                line["wait_inst_%"] = 100 * cs["SQ_WAIT_INST_ANY"] / wc
                line["active_%"] = 100 * cs["SQ_ACTIVE_INST_ANY"] / wc
            if cs.get("GRBM_GUI_ACTIVE"):
                # MFMA busy cycles are summed over all SIMDs (1024 on MI355X)
                line["mfma_busy_%"] = 100 * cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (
                    cs["GRBM_GUI_ACTIVE"] / 8 * 1024)
                line["eff_clock_GHz"] = cs["GRBM_GUI_ACTIVE"] / 8 / max(durs.get(k, 1), 1)
            if "SQ_LDS_BANK_CONFLICT" in cs:
                line["lds_bank_conflict_cyc"] = cs["SQ_LDS_BANK_CONFLICT"]
            if cs.get("TCC_HIT_sum") is not None and cs.get("TCC_MISS_sum") is not None:
                tot = cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]
                line["l2_hit_%"] = 100 * cs["TCC_HIT_sum"] / tot if tot else None
                rd = cs.get("TCC_EA0_RDREQ_sum", 0) * 64
                wr = cs.get("TCC_EA0_WRREQ_sum", 0) * 64
                line["ea_rd_MB"] = rd / 1e6
                line["ea_wr_MB"] = wr / 1e6
                if durs.get(k):
                    line["ea_TBps"] = (rd + wr) / durs[k] / 1e3
            out.append(line)
    for l in out:
        print({k: (round(v, 2) if isinstance(v, float) else v) for k, v in l.items()})
    return out


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
