"""Steady-state kernel table from a ``rocprofv3 --kernel-trace`` CSV.

A profiled training / forward run also contains its warmup (the GEMM autotuner times every
candidate, hipBLASLt included, on the first calls of each shape). This keeps only the
dispatches after the N-th completion of a marker kernel (e.g. the optimizer's AdamW kernel, 2 per
GPT-2 step with the split optimizer) and prints per kernel: calls, total / mean µs, share of the
window's GPU time, plus the share of hipBLASLt (``Cijk_*``) kernels.

The side-stream probes (parallel/streams.py: 1-workgroup ``spin`` kernels that check a side
stream still runs beside the compute stream) run during the warm-up and once after it, never in
the timed loop; the window starts after the LAST probe dispatch as well, and
``probes_in_window`` says whether any probe was still inside it.

Queue map: rocprofv3's kernel trace records the hardware queue (``Queue_Id``) and the HIP stream
(``Stream_Id``) of every dispatch. Two streams that were meant to overlap but show ONE queue id
execute in order (the stream-to-queue serialisation of profiles/r05_step/SUMMARY.md §12); the
``queues`` summary lists, per queue, the streams it served in the window and their busy time.

    python tools/prof_steady.py TRACE.csv --marker adamw_kernel --skip 6 [--csv OUT.csv]
"""

import argparse
import csv
import json
import sys
from collections import defaultdict


def _queue_map(win):
    """Per hardware queue: the streams it served and their busy time in the window."""
    if not win or "Queue_Id" not in win[0]:
        return None
    q = defaultdict(lambda: defaultdict(lambda: [0, 0]))
    for r in win:
        a = q[r["Queue_Id"]][r.get("Stream_Id", "?")]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return {qid: {sid: {"dispatches": v[0], "busy_ms": round(v[1] / 1e6, 3)}
                  for sid, v in streams.items()} for qid, streams in sorted(q.items())}


def steady(path, marker, skip, probe="spin"):
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
    probes = [r for r in rows if probe and probe in r["Kernel_Name"]]
    skipped_markers = 0
    if probes:
        # start after the last probe too; a probe after t0 is the post-warm-up re-check, and the
        # marker completions it pushes out of the window are reported
        t_probe = max(int(r["End_Timestamp"]) for r in probes)
        if t_probe > t0:
            skipped_markers = sum(1 for r in rows if marker in r["Kernel_Name"]
                                  and t0 < int(r["End_Timestamp"]) <= t_probe)
            t0 = t_probe
    win = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
    n_probe_win = sum(1 for r in win if probe and probe in r["Kernel_Name"])    # 0 by design
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
                 if total else None, "marker": marker, "skip": skip,
                 "probes_in_window": n_probe_win, "markers_skipped_for_probes": skipped_markers,
                 "queues": _queue_map(win)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", required=True)
    ap.add_argument("--skip", type=int, required=True)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--probe", default="spin",
                    help="name fragment of the side-stream probe kernel ('' = keep probes)")
    a = ap.parse_args()
    out, summ = steady(a.trace, a.marker, a.skip, a.probe)
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
