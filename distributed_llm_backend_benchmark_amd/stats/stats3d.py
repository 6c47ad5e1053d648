"""3D (activation-shaped) collective statistics.

Reproduces reference ``collectives/3d/stats.py``: ms statistics per file (32-49), records keyed
by implementation/op/ranks/hidden/seq/batch (90-110), a standard CSV with the same 12 columns
sorted op → ranks → hidden → seq → batch (146-185) and a transposed CSV with
``<op>_r<P>_h<H>_s<S>_b<B>`` column ids plus the metadata block (187-282).

Additions written to ``..._ext.csv``: ``tensor_size_bytes``, ``dtype``, ``wire_dtype``,
``rank_max_p50_ms``, ``algbw_gbps``/``busbw_gbps`` at p50 (nccl-tests convention on the bytes
actually put on the wire: the reference's MPI 3D path sent fp32 while labelling bf16 sizes,
SURVEY §2.8 item 3).
"""

from __future__ import annotations

import csv
import glob
import os
from typing import Dict, List

import numpy as np

from ..utils.io import load_json, save_json
from .bandwidth import algbw_gbps, busbw_gbps
from .stats1d import op_impl_label, rank_max_p50, refused

STANDARD_COLUMNS = [
    "implementation", "operation", "num_ranks", "hidden_dim", "seq_len", "batch",
    "tensor_size_mb", "num_elements", "mean_time_ms", "median_time_ms", "min_time_ms",
    "max_time_ms",
]
EXT_COLUMNS = STANDARD_COLUMNS + [
    "tensor_size_bytes", "dtype", "wire_dtype", "wire_bytes", "rank_max_p50_ms",
    "algbw_gbps", "busbw_gbps", "timing_method", "op_impl",
]
_METRICS = ["mean_time_ms", "median_time_ms", "min_time_ms", "max_time_ms"]


def calculate_statistics(timings_2d) -> Dict[str, float]:
    flat = np.asarray(timings_2d, dtype=np.float64).flatten()
    return {
        "mean_time_ms": float(np.mean(flat)) * 1e3,
        "median_time_ms": float(np.median(flat)) * 1e3,
        "min_time_ms": float(np.min(flat)) * 1e3,
        "max_time_ms": float(np.max(flat)) * 1e3,
    }


def stats_for_result(data: Dict[str, object]) -> Dict[str, object]:
    shp = data["tensor_shape"]
    p = int(data["num_ranks"])
    op = data["operation"]
    st = calculate_statistics(data["timings"])
    size_bytes = int(data.get("tensor_size_bytes") or int(data["num_elements"]) * 2)
    wire_dtype = data.get("wire_dtype", data.get("dtype", "bfloat16"))
    wire_bytes = int(data.get("wire_bytes") or size_bytes)
    p50 = st["median_time_ms"] / 1e3
    return {
        "implementation": data.get("mpi_implementation") or data.get("implementation"),
        "operation": op,
        "num_ranks": p,
        "hidden_dim": shp["hidden_dim"],
        "seq_len": shp["seq_len"],
        "batch": shp["batch"],
        "tensor_size_mb": round(float(data["tensor_size_mb"]), 4),
        "num_elements": data["num_elements"],
        **st,
        "tensor_size_bytes": size_bytes,
        "dtype": data.get("dtype", "bfloat16"),
        "wire_dtype": wire_dtype,
        "wire_bytes": wire_bytes,
        "rank_max_p50_ms": rank_max_p50(data["timings"]) * 1e3,
        "algbw_gbps": algbw_gbps(op, wire_bytes, p50, p),
        "busbw_gbps": busbw_gbps(op, wire_bytes, p50, p),
        "timing_method": data.get("timing_method"),
        "op_impl": op_impl_label(data),
    }


def _sorted(rows: List[Dict[str, object]]) -> List[Dict[str, object]]:
    return sorted(rows, key=lambda r: (r["operation"], r["num_ranks"], r["hidden_dim"],
                                       r["seq_len"], r["batch"]))


def write_standard_csv(path: str, rows: List[Dict[str, object]], columns=None) -> None:
    columns = columns or STANDARD_COLUMNS
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=columns, extrasaction="ignore")
        w.writeheader()
        for r in _sorted(rows):
            w.writerow({k: r.get(k) for k in columns})


def config_id(r: Dict[str, object]) -> str:
    return (f"{r['operation']}_r{r['num_ranks']}_h{r['hidden_dim']}_"
            f"s{r['seq_len']}_b{r['batch']}")


def write_transpose_csv(path: str, rows: List[Dict[str, object]]) -> None:
    rows = _sorted(rows)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Metric"] + [config_id(r) for r in rows])
        for m in _METRICS:
            w.writerow([m] + [r[m] for r in rows])
        w.writerow([])
        w.writerow(["--- Metadata ---"])
        for m in ("operation", "num_ranks", "hidden_dim", "seq_len", "batch", "tensor_size_mb"):
            w.writerow([m] + [r[m] for r in rows])


def process_directory(input_dir: str, output_dir: str, impl_label: str,
                      verbose: bool = True) -> List[Dict[str, object]]:
    """Reference ``process_implementation`` (``collectives/3d/stats.py:51-144``)."""
    os.makedirs(output_dir, exist_ok=True)
    rows: List[Dict[str, object]] = []
    for fp in sorted(glob.glob(os.path.join(input_dir, "*.json"))):
        if fp.endswith(".error.json"):
            continue
        try:
            data = load_json(fp)
            if "timings" not in data or "tensor_shape" not in data:
                continue
            why = refused(data)
            if why:
                if verbose:
                    print(f"  REFUSED {os.path.basename(fp)}: {why}")
                continue
            r = stats_for_result(data)
        except Exception as e:
            if verbose:
                print(f"  ERROR processing {os.path.basename(fp)}: {e}")
            continue
        stem = os.path.splitext(os.path.basename(fp))[0]
        save_json(r, os.path.join(output_dir, stem + "_stats.json"))
        rows.append(r)
    if rows:
        write_standard_csv(os.path.join(output_dir,
                           f"benchmark_statistics_3d_{impl_label}_standard.csv"), rows)
        write_transpose_csv(os.path.join(output_dir,
                            f"benchmark_statistics_3d_{impl_label}_transpose.csv"), rows)
        write_standard_csv(os.path.join(output_dir,
                           f"benchmark_statistics_3d_{impl_label}_ext.csv"), rows, EXT_COLUMNS)
    if verbose:
        print(f"Processed {len(rows)} 3D files from {input_dir} -> {output_dir}")
    return rows
