"""YAML experiment config with the reference schema.

Reference schema: ``config/baseline_config.yaml:1-34`` — sections ``experiment``, ``model``,
``parallelism``, ``input``, ``execution``, ``system``. Keys are read by the reference at
``run_mpi.py:73,82,100-110,154,172,237-238``, ``models.py:323-333``, ``data_gen.py:66-71``
and ``utils.py:163-169``.

Additions (all optional, defaults keep reference behaviour):

* ``parallelism.backend``: ``rccl`` | ``gloo`` | ``auto`` (process-group backend).
* ``parallelism.world_size: auto`` accepts whatever world the launcher created.
* ``parallelism.cores_per_rank`` is accepted and recorded; on GPU it is a no-op.
* ``execution.allreduce``: ``rccl`` (torch ProcessGroupNCCL) | ``native`` (our C++ RCCL engine
  on the compute stream) | ``custom`` (IPC xGMI kernel) | ``auto`` (custom below its crossover,
  native above) — the row-parallel all-reduce path.
* ``execution.allreduce_dtype``: ``bf16`` (on-device, default) | ``fp32`` (reference wire format,
  ``models.py:84``).
* ``execution.attention``: ``slice`` (reference stub ``models.py:162-167``) | ``sdpa``.
* ``execution.kernels``: ``hip`` (hand-written gfx950 kernels) | ``torch``.
* ``execution.overlap_chunks``: micro-batches the TP forward interleaves so each row-parallel
  all-reduce runs under another micro-batch's GEMMs (1 = the reference's blocking order).
"""

from __future__ import annotations

import copy
import os
from typing import Any, Dict

import yaml

DEFAULT_CONFIG: Dict[str, Any] = {
    "experiment": {"name": "baseline_7b_world4", "output_dir": "results"},
    "model": {
        "size": "7B",
        "hidden_size": 4096,
        "num_layers": 32,
        "num_heads": 32,
        "ffn_intermediate": 16384,
    },
    "parallelism": {"world_size": 4, "cores_per_rank": 14, "backend": "auto"},
    "input": {"batch_size": 8, "sequence_length": 512, "seed": 42},
    "execution": {
        "warmup_iterations": 5,
        "benchmark_iterations": 10,
        "allreduce": "auto",
        "allreduce_dtype": "bf16",
        "attention": "slice",
        "kernels": "hip",
        "overlap_chunks": 1,
    },
    "system": {"omp_num_threads": 14, "mkl_num_threads": 14},
}

REQUIRED_SECTIONS = ("experiment", "model", "parallelism", "input", "execution", "system")

_REQUIRED_KEYS = {
    "experiment": ("name", "output_dir"),
    "model": ("hidden_size", "num_layers", "num_heads", "ffn_intermediate"),
    "parallelism": ("world_size",),
    "input": ("batch_size", "sequence_length", "seed"),
    "execution": ("warmup_iterations", "benchmark_iterations"),
}


class ConfigError(ValueError):
    pass


def _merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = v
    return out


def validate_config(config: Dict[str, Any]) -> Dict[str, Any]:
    """Check the reference-required keys; fill optional additions with defaults."""
    if not isinstance(config, dict):
        raise ConfigError("config must be a mapping")
    for sec in REQUIRED_SECTIONS[:-1]:
        if sec not in config:
            raise ConfigError(f"missing config section '{sec}'")
        for key in _REQUIRED_KEYS.get(sec, ()):
            if key not in config[sec]:
                raise ConfigError(f"missing config key '{sec}.{key}'")
    cfg = _merge({k: {} for k in REQUIRED_SECTIONS}, config)
    for sec in ("parallelism", "execution"):
        for k, v in DEFAULT_CONFIG[sec].items():
            cfg[sec].setdefault(k, v)
    cfg["model"].setdefault("size", "custom")
    ws = cfg["parallelism"]["world_size"]
    if ws != "auto" and (not isinstance(ws, int) or ws < 1):
        raise ConfigError(f"parallelism.world_size must be a positive int or 'auto', got {ws!r}")
    m = cfg["model"]
    for k in ("hidden_size", "num_layers", "num_heads", "ffn_intermediate"):
        if int(m[k]) <= 0:
            raise ConfigError(f"model.{k} must be positive")
    ex = cfg["execution"]
    if ex["allreduce"] not in ("auto", "rccl", "custom", "native", "torch", "emulate"):
        raise ConfigError("execution.allreduce must be auto|rccl|custom|native|torch, got "
                          f"{ex['allreduce']!r}")
    if ex["allreduce_dtype"] not in ("bf16", "fp32"):
        raise ConfigError("execution.allreduce_dtype must be bf16|fp32")
    if ex["attention"] not in ("slice", "sdpa"):
        raise ConfigError("execution.attention must be slice|sdpa")
    if ex["kernels"] not in ("hip", "torch"):
        raise ConfigError("execution.kernels must be hip|torch")
    if not isinstance(ex["overlap_chunks"], int) or ex["overlap_chunks"] < 1:
        raise ConfigError("execution.overlap_chunks must be a positive int")
    return cfg


def load_config(config_path: str) -> Dict[str, Any]:
    """``yaml.safe_load`` + schema validation (reference ``utils.py:90-102``)."""
    with open(config_path, "r") as f:
        raw = yaml.safe_load(f)
    return validate_config(raw)


def setup_environment(config: Dict[str, Any]) -> None:
    """Export OMP/MKL thread counts (reference ``utils.py:154-169``).

    The reference sets these *after* ``import torch``, which is too late
    for the OpenMP runtime; our CLIs call this before importing torch.
    """
    sysc = config.get("system", {}) or {}
    if "omp_num_threads" in sysc:
        os.environ["OMP_NUM_THREADS"] = str(sysc["omp_num_threads"])
    if "mkl_num_threads" in sysc:
        os.environ["MKL_NUM_THREADS"] = str(sysc["mkl_num_threads"])
