"""Result-file schema and names (the reference's "results layout").

1D: ``<impl>_<op>_ranks<P>_<sizeName>.json`` (reference ``collectives/1d/openmpi.py:288``,
``collectives/1d/dsccl.py:251``) with keys ``implementation, backend, operation, num_ranks,
data_size_name, num_elements, dtype, warmup_iterations, measurement_iterations,
timing_method, timings`` (``1d/dsccl.py:237-249``; the MPI variant's ``mpi_implementation``
key is written too so both reference stats readers accept it).

3D: ``<impl>_<op>_ranks<P>_b<B>_s<S>_h<H>.json`` (``collectives/3d/dsccl.py:227``) adding
``tensor_shape{batch,seq_len,hidden_dim}``, ``tensor_size_bytes``, ``tensor_size_mb``
(``3d/dsccl.py:207-225``).

Additions: ``bytes`` (true message bytes; the reference's 1D labels are 2x the real size,
SURVEY §2.8 item 1), ``host_timings``, ``batched_mean_s``, ``wire_dtype``/``wire_bytes``,
``validated``, ``device``, ``env``.
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional

# reference labels -> fp16 element counts (collectives/1d/openmpi.py:23-28)
REFERENCE_1D_SIZES: "OrderedDict[str, int]" = OrderedDict(
    [("1KB", 256), ("64KB", 16384), ("1MB", 262144), ("16MB", 4194304)])

REFERENCE_3D_BATCH = [1, 8, 16, 32]        # collectives/3d/openmpi.py:21
REFERENCE_3D_SEQ = [1, 2048, 4096, 8192]   # collectives/3d/openmpi.py:22
REFERENCE_3D_HIDDEN = [2048, 4096]         # collectives/3d/openmpi.py:23


def bytes_label(nbytes: int) -> str:
    for unit, div in (("GiB", 1 << 30), ("MiB", 1 << 20), ("KiB", 1 << 10)):
        if nbytes >= div and nbytes % div == 0:
            return f"{nbytes // div}{unit}"
    return f"{nbytes}B"


def parse_bytes(text: str) -> int:
    t = text.strip()
    mult = {"B": 1, "K": 1 << 10, "KB": 1 << 10, "KIB": 1 << 10, "M": 1 << 20, "MB": 1 << 20,
            "MIB": 1 << 20, "G": 1 << 30, "GB": 1 << 30, "GIB": 1 << 30}
    num = ""
    i = 0
    while i < len(t) and (t[i].isdigit() or t[i] == "."):
        num += t[i]
        i += 1
    unit = t[i:].strip().upper() or "B"
    if unit not in mult:
        raise ValueError(f"bad size {text!r}")
    return int(float(num) * mult[unit])


def sweep_sizes(min_bytes: int, max_bytes: int, elem_size: int,
                factor: int = 2) -> "OrderedDict[str, int]":
    out: "OrderedDict[str, int]" = OrderedDict()
    b = max(min_bytes, elem_size)
    while b <= max_bytes:
        out[bytes_label(b)] = b // elem_size
        b *= factor
    return out


def resolve_1d_sizes(spec: str, elem_size: int) -> "OrderedDict[str, int]":
    """``reference`` | ``sweep`` (1 KiB..1 GiB ×2) | ``LO:HI`` range | comma list of byte sizes."""
    spec = (spec or "reference").strip()
    if spec == "reference":
        return OrderedDict(REFERENCE_1D_SIZES)
    if spec == "sweep":
        return sweep_sizes(1 << 10, 1 << 30, elem_size)
    if ":" in spec:
        lo, hi = spec.split(":", 1)
        return sweep_sizes(parse_bytes(lo), parse_bytes(hi), elem_size)
    out: "OrderedDict[str, int]" = OrderedDict()
    for tok in spec.split(","):
        tok = tok.strip()
        if tok in REFERENCE_1D_SIZES:
            out[tok] = REFERENCE_1D_SIZES[tok]
        else:
            b = parse_bytes(tok)
            out[bytes_label(b)] = max(1, b // elem_size)
    return out


def filename_1d(impl: str, op: str, ranks: int, size_name: str) -> str:
    return f"{impl}_{op}_ranks{ranks}_{size_name}.json"


def filename_3d(impl: str, op: str, ranks: int, b: int, s: int, h: int) -> str:
    return f"{impl}_{op}_ranks{ranks}_b{b}_s{s}_h{h}.json"


def result_1d(*, impl: str, backend: str, op: str, ranks: int, size_name: str,
              num_elements: int, dtype: str, nbytes: int, warmup: int, iters: int,
              timing_method: str, timings: List[List[float]],
              host_timings: Optional[List[List[float]]] = None,
              batched_mean_s: Optional[float] = None, extra: Optional[Dict] = None) -> Dict:
    res = {
        "implementation": impl,
        "mpi_implementation": impl,
        "backend": backend,
        "operation": op,
        "num_ranks": ranks,
        "data_size_name": size_name,
        "num_elements": num_elements,
        "dtype": dtype,
        "bytes": nbytes,
        "warmup_iterations": warmup,
        "measurement_iterations": iters,
        "timing_method": timing_method,
        "timings": timings,
    }
    if host_timings is not None:
        res["host_timings"] = host_timings
    if batched_mean_s is not None:
        res["batched_mean_s"] = batched_mean_s
    if extra:
        res.update(extra)
    return res


def result_3d(*, impl: str, backend: str, op: str, ranks: int, batch: int, seq_len: int,
              hidden_dim: int, dtype: str, wire_dtype: str, wire_bytes: int, warmup: int,
              iters: int, timing_method: str, timings: List[List[float]],
              host_timings: Optional[List[List[float]]] = None,
              batched_mean_s: Optional[float] = None, extra: Optional[Dict] = None) -> Dict:
    n = batch * seq_len * hidden_dim
    size_bytes = n * 2  # bf16 nominal size, as the reference labels it (3d/dsccl.py:161)
    res = {
        "implementation": impl,
        "backend": backend,
        "operation": op,
        "num_ranks": ranks,
        "tensor_shape": {"batch": batch, "seq_len": seq_len, "hidden_dim": hidden_dim},
        "num_elements": n,
        "tensor_size_bytes": size_bytes,
        "tensor_size_mb": size_bytes / (1024 * 1024),
        "dtype": dtype,
        "wire_dtype": wire_dtype,
        "wire_bytes": wire_bytes,
        "warmup_iterations": warmup,
        "measurement_iterations": iters,
        "timing_method": timing_method,
        "timings": timings,
    }
    if host_timings is not None:
        res["host_timings"] = host_timings
    if batched_mean_s is not None:
        res["batched_mean_s"] = batched_mean_s
    if extra:
        res.update(extra)
    return res
