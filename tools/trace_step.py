"""Per-kernel breakdown of ONE training step from a rocprofv3 kernel trace.

Steps are delimited by a marker kernel (default: the AdamW update); the last complete step is
summarised (time per kernel name, summed; gaps between kernels reported as idle).

    python tools/trace_step.py gpurun_out/prof_gpt2/gpt2_kernel_trace.csv [--marker adamw]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = ends[-2] + 1, ends[-1] + 1
    step = rows[lo:hi]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in step:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]][0] += 1
        agg[r["Kernel_Name"]][1] += d
        busy += d
    span = t1 - t0
    print(f"step span {span/1e3:.1f} us, kernel busy {busy/1e3:.1f} us, "
          f"idle {100*(span-busy)/span:.1f}%, {len(step)} kernels")
    for name, (n, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{d/1e3:9.1f} us {100*d/busy:5.1f}% x{n:4d}  {name[:110]}")


if __name__ == "__main__":
    main()
