"""Per-kernel mean PMC counter values from rocprofv3 ``--pmc`` runs (``*_counter_collection.csv``)
joined with the kernel-trace mean duration: one JSON line per (run dir, kernel).

    python tools/pmc_summary.py gpurun_out/pmc_lmhead_p1 gpurun_out/pmc_lmhead_p2 ... [--match S]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def summarize(d, match=None):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = []
    for f in cc:
        vals = defaultdict(lambda: defaultdict(list))
        dur = defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if "Start_Timestamp" in r and r.get("End_Timestamp"):
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, cs in vals.items():
            n = max(len(v) for v in cs.values())
            rec = {"dir": os.path.basename(d.rstrip("/")), "kernel": k[:90], "dispatch_rows": n}
            for c, v in cs.items():
                rec[c] = sum(v) / len(v)
            out.append(rec)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default=None)
    a = ap.parse_args()
    for d in a.dirs:
        for rec in summarize(d, a.match):
            print(json.dumps(rec))


if __name__ == "__main__":
    main()
