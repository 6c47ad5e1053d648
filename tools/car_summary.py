"""Markdown summary of tools/car_harness.py results (best workgroup count per configuration).

usage: python tools/car_summary.py profiles/r02_car_harness/*.jsonl > SUMMARY.md
"""

from __future__ import annotations

import json
import sys
from collections import defaultdict


def _size(n: int) -> str:
    return f"{n >> 20} MiB" if n >= 1 << 20 else f"{n >> 10} KiB" if n >= 1024 else f"{n} B"


def load(paths):
    rows = []
    for p in paths:
        with open(p) as f:
            rows += [json.loads(line) for line in f if line.strip()]
    return rows


def best(rows, section):
    out = {}
    for r in rows:
        if r.get("section") != section or not r.get("valid") or "us_b2b" not in r:
            continue
        k = (r["kind"], r["world"], r["bytes"])
        if k not in out or r["us_b2b"] < out[k]["us_b2b"]:
            out[k] = r
    return out


def main(paths) -> int:
    rows = load(paths)
    bad = [r for r in rows if not r.get("valid", True)]
    print(f"{len(rows)} configurations, {len(bad)} failed validation "
          "(each validated against an fp32 sum of the W rank inputs before timing).\n")
    lat = best(rows, "latency")
    if lat:
        print("## One-shot all-reduce latency (us per call, back to back; best workgroups/rank)\n")
        worlds = sorted({k[1] for k in lat})
        print("| message | " + " | ".join(f"W={w}" for w in worlds) + " |")
        print("|---|" + "---|" * len(worlds))
        for n in sorted({k[2] for k in lat}):
            cells = [f"{lat[('oneshot', w, n)]['us_b2b']:.2f} (p50 "
                     f"{lat[('oneshot', w, n)]['us_p50']:.2f})" if ('oneshot', w, n) in lat
                     else "-" for w in worlds]
            print(f"| {_size(n)} | " + " | ".join(cells) + " |")
        print()
    for sec, title in (("crossover", "One-shot vs staged two-shot vs registered two-shot"),
                       ("throughput", "Large-message all-reduce"),
                       ("direct", "Direct one-hop collectives (registered inputs)")):
        b = best(rows, sec)
        if not b:
            continue
        print(f"## {title} (us per call; GB/s = modelled bytes loaded + stored by all W ranks "
              "/ time — small messages are served from L2 / MALL, so it can exceed HBM peak)\n")
        kinds = sorted({k[0] for k in b})
        print("| W | message/rank | " + " | ".join(kinds) + " |")
        print("|---|---|" + "---|" * len(kinds))
        for w in sorted({k[1] for k in b}):
            for n in sorted({k[2] for k in b if k[1] == w}):
                cells = []
                for kd in kinds:
                    r = b.get((kd, w, n))
                    cells.append(f"{r['us_b2b']:.1f} ({r['hbm_GBps']:.0f} GB/s, nb {r['nblocks']})"
                                 if r else "-")
                print(f"| {w} | {_size(n)} | " + " | ".join(cells) + " |")
        print()
    st = [r for r in rows if r.get("section") == "streams"]
    if st:
        print("## Per-rank launches on W streams (production launch path, W concurrent kernels)\n")
        print("| W | kind | message | valid | host us/call |")
        print("|---|---|---|---|---|")
        for r in st:
            print(f"| {r['world']} | {r['kind']} | {_size(r['bytes'])} | {r['valid']} | "
                  f"{r.get('us_host_per_call', '-')} |")
        print()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
