"""Our results vs the reference's published statistics (the BASELINE comparison table).

The reference publishes numbers only as stats CSVs (``collectives/1d/stats/<impl>/
benchmark_statistics.csv`` with 14 columns, ``collectives/3d/stats/<impl>/
benchmark_statistics_3d_<impl>_standard.csv``; BASELINE.md cites their rows). This module joins
any of those with ours on the configuration key and reports, per configuration, the reference's
best p50 (over the given implementations), ours, the speedup and both busBW values:

* 1D key ``(operation, num_ranks, data_size_name)``; bytes = ``num_elements`` x element size
  (reference 1D data is fp16, ``collectives/1d/openmpi.py:23-28``: the "1KB" label is 512 B).
* 3D key ``(operation, num_ranks, batch, seq_len, hidden_dim)``; bytes = ``num_elements`` x 2
  (the tensors are bf16; BASELINE.md computes busBW from these bytes).

busBW uses the nccl-tests factors of :mod:`.bandwidth` at the p50 latency.
"""

from __future__ import annotations

import csv
import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .bandwidth import busbw_gbps

Key = Tuple


def _read(path: str) -> List[Dict[str, str]]:
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _elem_bytes(row: Dict[str, str], default: int) -> int:
    dt = (row.get("dtype") or "").lower()
    if dt in ("float32", "fp32"):
        return 4
    if dt in ("float16", "fp16", "bfloat16", "bf16"):
        return 2
    return default


def _impl(row: Dict[str, str], col: str) -> str:
    """Row label: the run's impl name, plus what actually ran when the stats ext CSV records it
    and it differs (``rccl[native_oop]``: the P = 1 out-of-place substitute)."""
    impl = row.get(col) or "?"
    op_impl = row.get("op_impl") or ""
    return f"{impl}[{op_impl}]" if op_impl and op_impl != impl else impl


def load_1d(paths: Iterable[str], default_elem_bytes: int = 2) -> Dict[Key, Dict[str, object]]:
    """Best (lowest p50) row per 1D key across the given stats CSVs."""
    best: Dict[Key, Dict[str, object]] = {}
    for p in paths:
        for r in _read(p):
            key = (r["operation"], int(r["num_ranks"]), r["data_size_name"])
            p50_us = float(r["median_time_us"])
            nbytes = int(r.get("bytes") or 0) or int(r["num_elements"]) * _elem_bytes(
                r, default_elem_bytes)
            rec = {"impl": _impl(r, "mpi_implementation"), "p50_us": p50_us, "bytes": nbytes}
            if key not in best or p50_us < best[key]["p50_us"]:
                best[key] = rec
    return best


def load_3d(paths: Iterable[str]) -> Dict[Key, Dict[str, object]]:
    best: Dict[Key, Dict[str, object]] = {}
    for p in paths:
        for r in _read(p):
            key = (r["operation"], int(r["num_ranks"]), int(r["batch"]), int(r["seq_len"]),
                   int(r["hidden_dim"]))
            p50_us = float(r["median_time_ms"]) * 1e3
            nbytes = int(r.get("tensor_size_bytes") or 0) or int(r["num_elements"]) * 2
            rec = {"impl": _impl(r, "implementation"), "p50_us": p50_us, "bytes": nbytes}
            if key not in best or p50_us < best[key]["p50_us"]:
                best[key] = rec
    return best


def compare(ours: Dict[Key, Dict[str, object]], ref: Dict[Key, Dict[str, object]],
            match_ranks: bool = True) -> List[Dict[str, object]]:
    """One row per configuration present in both. With ``match_ranks=False`` our results at any
    rank count are compared with the reference at the same key minus ranks (e.g. our world-1
    numbers against every reference P), labelled with both rank counts."""
    rows = []
    if match_ranks:
        pairs = [(k, k) for k in ours if k in ref]
    else:
        pairs = [(ko, kr) for ko in ours for kr in ref
                 if ko[0] == kr[0] and ko[2:] == kr[2:]]
    for ko, kr in sorted(pairs, key=lambda p: (str(p[1][0]), p[1][1:])):
        o, r = ours[ko], ref[kr]
        P = int(kr[1])
        Po = int(ko[1])
        o_bus = busbw_gbps(ko[0], int(o["bytes"]), o["p50_us"] * 1e-6, Po)
        r_bus = busbw_gbps(kr[0], int(r["bytes"]), r["p50_us"] * 1e-6, P)
        rows.append({
            "operation": kr[0], "ref_num_ranks": P, "our_num_ranks": Po,
            "config": "/".join(str(x) for x in kr[2:]),
            "ref_impl": r["impl"], "ref_p50_us": r["p50_us"], "ref_busbw_gbps": r_bus,
            "our_impl": o["impl"], "our_p50_us": o["p50_us"], "our_busbw_gbps": o_bus,
            "speedup_p50": (r["p50_us"] / o["p50_us"]) if o["p50_us"] > 0 else None,
        })
    return rows


COLUMNS = ["operation", "ref_num_ranks", "our_num_ranks", "config", "ref_impl", "ref_p50_us",
           "ref_busbw_gbps", "our_impl", "our_p50_us", "our_busbw_gbps", "speedup_p50"]


def write_csv(rows: Sequence[Dict[str, object]], path: str) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLUMNS)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def markdown(rows: Sequence[Dict[str, object]], limit: Optional[int] = None) -> str:
    head = ("| op | P ref / ours | config | ref impl | ref p50 µs | ref busBW | ours p50 µs | "
            "ours busBW | speedup |\n|---|---|---|---|---|---|---|---|---|\n")
    lines = []
    f2 = lambda v: "-" if v is None else f"{v:.2f}"   # noqa: E731
    for r in rows[:limit] if limit else rows:
        sp = r["speedup_p50"]
        lines.append(f"| {r['operation']} | {r['ref_num_ranks']} / {r['our_num_ranks']} | "
                     f"{r['config']} | {r['ref_impl']} | {r['ref_p50_us']:.1f} | "
                     f"{f2(r['ref_busbw_gbps'])} | {r['our_p50_us']:.1f} | "
                     f"{f2(r['our_busbw_gbps'])} | {'-' if sp is None else f'{sp:.1f}x'} |")
    return head + "\n".join(lines) + "\n"
