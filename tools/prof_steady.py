"""Steady-state kernel table from a ``rocprofv3 --kernel-trace`` CSV.

A profiled training / forward run also contains its warmup (the GEMM autotuner times every
candidate, hipBLASLt included, on the first calls of each shape). This keeps only the
dispatches after the N-th completion of a marker kernel (e.g. the optimizer's AdamW kernel, 2 per
GPT-2 step with the split optimizer) and prints per kernel: calls, total / mean µs, share of the
window's GPU time, plus the share of hipBLASLt (``Cijk_*``) kernels.

    python tools/prof_steady.py TRACE.csv --marker adamw_kernel --skip 6 [--csv OUT.csv]
"""

import argparse
import csv
import json
import sys
from collections import defaultdict


def steady(path, marker, skip):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = None
    seen = 0
    for r in rows:
        if marker in r["Kernel_Name"]:
            seen += 1
            if seen == skip:
                t0 = int(r["End_Timestamp"])
                break
    if t0 is None:
        raise SystemExit(f"marker {marker!r} seen {seen} times, fewer than --skip {skip}")
    win = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
    agg = defaultdict(lambda: [0, 0])
    for r in win:
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    total = sum(v[1] for v in agg.values())
    span = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"]) if win else 0
    out = [{"name": k, "calls": v[0], "total_us": v[1] / 1e3, "mean_us": v[1] / v[0] / 1e3,
            "pct": 100.0 * v[1] / total} for k, v in agg.items()]
    out.sort(key=lambda d: -d["total_us"])
    cijk = sum(d["total_us"] for d in out if "Cijk" in d["name"])
    return out, {"window_dispatches": len(win), "gpu_time_ms": total / 1e6,
                 "window_wall_ms": span / 1e6, "cijk_pct": round(100 * cijk * 1e3 / total, 2)
                 if total else None, "marker": marker, "skip": skip}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", required=True)
    ap.add_argument("--skip", type=int, required=True)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    out, summ = steady(a.trace, a.marker, a.skip)
    print(json.dumps(summ))
    for d in out[:a.top]:
        print(f"{d['pct']:6.2f}%  {d['calls']:6d}  {d['mean_us']:9.2f} us  {d['name'][:110]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["name", "calls", "total_us", "mean_us", "pct"])
            w.writeheader()
            for d in out:
                w.writerow({k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()})
            f.write(f"# {json.dumps(summ)}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
