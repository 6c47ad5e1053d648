"""1D collective statistics.

Reproduces reference ``collectives/1d/stats.py``:

* ``calculate_statistics`` (reference 26-75): flatten ``[rank][iter]`` seconds and report
  mean/median/min/max/std/p95/p99 in µs, per-rank means, load imbalance
  ``(max per-rank mean - mean of means) / mean of means * 100``.
* ``bandwidth_gbps`` = the reference's legacy formula evaluated at the flattened MAX time
  (reference 176-185).
* Per-file ``<stem>_stats.json`` and ``benchmark_statistics.csv`` with the same 14 columns in the
  same order (reference 226-241).

Additions: ``bytes``, ``algbw_gbps``/``busbw_gbps`` at the p50 latency (nccl-tests convention,
:mod:`.bandwidth`), ``rank_max_p50_us`` (median over iterations of the per-iteration max over
ranks — the number that bounds a synchronous collective) written to
``benchmark_statistics_ext.csv``; and a transposed CSV (the commented-out variant at reference
252-274 that produced the committed ``*_chng.csv``).
"""

from __future__ import annotations

import csv
import glob
import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..utils.io import load_json, save_json
from .bandwidth import (KNOWN_OPS, algbw_gbps, busbw_gbps, legacy_bandwidth_gbps,
                        roofline_violation)

LEGACY_COLUMNS = [
    "mpi_implementation", "operation", "num_ranks", "data_size_name", "num_elements",
    "mean_time_us", "median_time_us", "min_time_us", "max_time_us", "std_dev_us",
    "p95_time_us", "p99_time_us", "load_imbalance_percent", "bandwidth_gbps",
]

EXT_COLUMNS = LEGACY_COLUMNS + [
    "dtype", "bytes", "rank_max_p50_us", "algbw_gbps", "busbw_gbps", "timing_method",
    "op_impl",
]


def op_impl_label(data: Dict[str, object]) -> str:
    """What actually ran: the op implementation recorded by the sweep, with the
    out-of-place substitution marked — at P = 1 an in-place all-reduce / broadcast / reduce
    enqueues nothing, so the sweep times our native engine's out-of-place form under the
    run's impl directory; this label keeps such rows from being read as ProcessGroupNCCL."""
    impl = str(data.get("op_impl") or data.get("implementation") or
               data.get("mpi_implementation") or "")
    return impl + ("_oop" if data.get("out_of_place") else "")

_DTYPE_BYTES = {
    "float16": 2, "fp16": 2, "<class 'numpy.float16'>": 2, "bfloat16": 2, "bf16": 2,
    "float32": 4, "fp32": 4, "<class 'numpy.float32'>": 4, "float64": 8,
}


def dtype_nbytes(dtype: str) -> int:
    return _DTYPE_BYTES.get(str(dtype), 2)


def calculate_statistics(timings_2d: Sequence[Sequence[float]]) -> Dict[str, object]:
    arr = np.asarray(timings_2d, dtype=np.float64)
    if arr.ndim == 1:
        arr = arr[None, :]
    per_rank_means = np.mean(arr, axis=1)
    flat = arr.flatten()
    mean_of_means = float(np.mean(per_rank_means))
    imb = ((float(np.max(per_rank_means)) - mean_of_means) / mean_of_means * 100.0
           if mean_of_means > 0 else 0.0)
    return {
        "mean_time_us": float(np.mean(flat)) * 1e6,
        "median_time_us": float(np.median(flat)) * 1e6,
        "min_time_us": float(np.min(flat)) * 1e6,
        "max_time_us": float(np.max(flat)) * 1e6,
        "std_dev_us": float(np.std(flat)) * 1e6,
        "p95_time_us": float(np.percentile(flat, 95)) * 1e6,
        "p99_time_us": float(np.percentile(flat, 99)) * 1e6,
        "load_imbalance_percent": imb,
        "per_rank_means_us": (per_rank_means * 1e6).tolist(),
    }


def rank_max_p50(timings_2d: Sequence[Sequence[float]]) -> float:
    """Median over iterations of max over ranks, seconds."""
    arr = np.asarray(timings_2d, dtype=np.float64)
    if arr.ndim == 1:
        return float(np.median(arr))
    n = min(len(r) for r in timings_2d)
    arr = np.asarray([r[:n] for r in timings_2d], dtype=np.float64)
    return float(np.median(np.max(arr, axis=0)))


def refused(data: Dict[str, object]) -> Optional[str]:
    """Why a raw result must not become a statistic (None: fine): flagged invalid by the sweep,
    failed its closed-form validation (``validated: false``), or its p50 below the memory / xGMI roofline (``stats.bandwidth``) — an empty call, e.g. an
    in-place collective at one rank."""
    if data.get("invalid"):
        return str(data["invalid"])
    if data.get("validated") is False:      # a collective that returned a wrong result
        return "wrong_result"
    flat = [x for row in data["timings"] for x in (row if isinstance(row, list) else [row])]
    if not flat:
        return "no timings"
    nbytes = data.get("bytes") or data.get("wire_bytes") or data.get("tensor_size_bytes")
    if nbytes is None:
        nbytes = int(data["num_elements"]) * dtype_nbytes(str(data.get("dtype", "float16")))
    op = data["operation"]
    if op not in KNOWN_OPS:
        return None
    return roofline_violation(op, float(nbytes), float(np.median(flat)), int(data["num_ranks"]),
                              bool(data.get("colocated", False)))


def stats_for_result(data: Dict[str, object]) -> Dict[str, object]:
    impl = data.get("mpi_implementation") or data.get("implementation") or "unknown"
    op = data["operation"]
    p = int(data["num_ranks"])
    n = int(data["num_elements"])
    dtype = data.get("dtype", "float16")
    timings = data["timings"]
    st = calculate_statistics(timings)
    st["bandwidth_gbps"] = legacy_bandwidth_gbps(n, st["max_time_us"] / 1e6, p, op)
    nbytes = int(data.get("bytes") or n * dtype_nbytes(dtype))
    p50 = st["median_time_us"] / 1e6
    out = {
        "mpi_implementation": impl,
        "operation": op,
        "num_ranks": p,
        "data_size_name": data["data_size_name"],
        "num_elements": n,
        "dtype": dtype,
        **st,
        "bytes": nbytes,
        "rank_max_p50_us": rank_max_p50(timings) * 1e6,
        "algbw_gbps": algbw_gbps(op, nbytes, p50, p),
        "busbw_gbps": busbw_gbps(op, nbytes, p50, p),
        "timing_method": data.get("timing_method", "MPI.Wtime()"),
        "op_impl": op_impl_label(data),
    }
    return out


def _write_csv(path: str, columns: List[str], rows: List[Dict[str, object]]) -> None:
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=columns, extrasaction="ignore")
        w.writeheader()
        for r in rows:
            w.writerow({k: r.get(k) for k in columns})


def write_transposed_csv(path: str, rows: List[Dict[str, object]],
                         columns: Optional[List[str]] = None) -> None:
    columns = columns or [c for c in LEGACY_COLUMNS]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["metric"] + [f"run_{i + 1}" for i in range(len(rows))])
        for m in columns:
            w.writerow([m] + [r.get(m, "") for r in rows])


def process_directory(input_dir: str, output_dir: str,
                      csv_name: str = "benchmark_statistics.csv",
                      verbose: bool = True) -> List[Dict[str, object]]:
    """Reference ``process_all_json_files`` (``collectives/1d/stats.py:135-288``)."""
    os.makedirs(output_dir, exist_ok=True)
    files = sorted(glob.glob(os.path.join(input_dir, "*.json")))
    files = [f for f in files if not f.endswith(".error.json")]
    results: List[Dict[str, object]] = []
    for fp in files:
        try:
            data = load_json(fp)
            if "timings" not in data:
                continue
            why = refused(data)
            if why:
                if verbose:
                    print(f"  REFUSED {os.path.basename(fp)}: {why}")
                continue
            res = stats_for_result(data)
        except Exception as e:  # reference: print + continue (stats.py:215-217)
            if verbose:
                print(f"  ERROR processing {os.path.basename(fp)}: {e}")
            continue
        stem = os.path.splitext(os.path.basename(fp))[0]
        save_json(res, os.path.join(output_dir, stem + "_stats.json"))
        results.append(res)
    if results:
        _write_csv(os.path.join(output_dir, csv_name), LEGACY_COLUMNS, results)
        base, ext = os.path.splitext(csv_name)
        _write_csv(os.path.join(output_dir, base + "_ext" + ext), EXT_COLUMNS, results)
        write_transposed_csv(os.path.join(output_dir, base + "_transpose" + ext), results)
    if verbose:
        print(f"Processed {len(results)} files from {input_dir} -> {output_dir}")
    return results
