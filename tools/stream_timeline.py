"""Per-stream timeline of training steps from a ``rocprofv3 --kernel-trace`` CSV.

For the last ``--steps`` complete steps (delimited by the N-th completion of a marker kernel,
default the AdamW update: 2 per GPT-2 step with the split optimizer, so ``--per-step 2``):
wall time, per queue/stream the busy time (union of its kernels' intervals), the time with
kernels of two or more streams running at once, the time with NO kernel running (launch gaps,
host waits), and the top kernels of each stream by summed duration. Answers "which stream is the
critical path, and how much of the step is idle" — the question behind eager vs graph replay
and the side-stream weight gradients.

    python tools/stream_timeline.py TRACE.csv [--marker adamw_kernel --per-step 2 --steps 3]
"""

import argparse
import collections
import csv
import json


def _union(iv):
    """Total length of the union of [a, b) intervals."""
    tot, cur_a, cur_b = 0, None, None
    for a, b in sorted(iv):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def _coverage(iv_by_stream, t0, t1):
    """(ns with >= 1 stream busy, ns with >= 2 streams busy) inside [t0, t1)."""
    ev = []
    for sid, iv in iv_by_stream.items():
        merged = []
        for a, b in sorted(iv):
            a, b = max(a, t0), min(b, t1)
            if b <= a:
                continue
            if merged and a <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], b)
            else:
                merged.append([a, b])
        for a, b in merged:
            ev += [(a, 1), (b, -1)]
    ev.sort()
    busy1 = busy2 = 0
    depth, last = 0, None
    for t, d in ev:
        if last is not None and depth >= 1:
            busy1 += t - last
            if depth >= 2:
                busy2 += t - last
        depth += d
        last = t
    return busy1, busy2


def analyse(path, marker="adamw_kernel", per_step=2, steps=3, top=6):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sid_col = next((c for c in ("Stream_Id", "Queue_Id") if c in rows[0]), None)
    marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    ends = marks[per_step - 1::per_step]
    if len(ends) < steps + 1:
        raise SystemExit(f"only {len(ends)} step ends found for marker {marker!r}")
    out = []
    for k in range(len(ends) - steps, len(ends)):
        t0 = int(rows[ends[k - 1]]["End_Timestamp"])
        t1 = int(rows[ends[k]]["End_Timestamp"])
        ivs = collections.defaultdict(list)
        per_kernel = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in rows:
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if b <= t0 or a >= t1:
                continue
            sid = r.get(sid_col, "0") if sid_col else "0"
            ivs[sid].append((a, b))
            per_kernel[sid][r["Kernel_Name"][:90]] += (min(b, t1) - max(a, t0)) / 1e3
        busy1, busy2 = _coverage(ivs, t0, t1)
        streams = {}
        for sid, iv in ivs.items():
            clipped = [(max(a, t0), min(b, t1)) for a, b in iv]
            kt = sorted(per_kernel[sid].items(), key=lambda kv: -kv[1])[:top]
            streams[sid] = {"kernels": len(iv), "busy_us": round(_union(clipped) / 1e3, 1),
                            "top_us": {n: round(v, 1) for n, v in kt}}
        out.append({"wall_us": round((t1 - t0) / 1e3, 1),
                    "any_busy_us": round(busy1 / 1e3, 1),
                    "idle_us": round((t1 - t0 - busy1) / 1e3, 1),
                    "overlap_2plus_us": round(busy2 / 1e3, 1),
                    "stream_column": sid_col, "streams": streams})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_kernel")
    ap.add_argument("--per-step", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    for s in analyse(a.trace, a.marker, a.per_step, a.steps, a.top):
        print(json.dumps(s))


if __name__ == "__main__":
    main()
