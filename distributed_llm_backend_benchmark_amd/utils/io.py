"""JSON IO (reference ``utils.py:105-129``, ``utils.py:268-279``)."""

from __future__ import annotations

import json
import math
import os
from pathlib import Path
from typing import Any


def _sanitize(obj: Any) -> Any:
    """Make numpy scalars / NaN JSON-safe (NaN -> None)."""
    try:
        import numpy as np
    except Exception:  # pragma: no cover
        np = None
    if isinstance(obj, dict):
        return {str(k): _sanitize(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_sanitize(v) for v in obj]
    if np is not None:
        if isinstance(obj, np.generic):
            obj = obj.item()
        elif isinstance(obj, np.ndarray):
            return _sanitize(obj.tolist())
    if isinstance(obj, float) and (math.isnan(obj) or math.isinf(obj)):
        return None
    return obj


def save_json(data: Any, filepath: str, indent: int = 2) -> None:
    """Atomic write: tmp file + rename, so an interrupted sweep never leaves a truncated
    result that ``--resume`` would then skip."""
    path = Path(filepath)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + f".tmp{os.getpid()}")
    with open(tmp, "w") as f:
        json.dump(_sanitize(data), f, indent=indent)
    os.replace(tmp, path)


def load_json(filepath: str) -> Any:
    with open(filepath, "r") as f:
        return json.load(f)


def save_results(results: Any, output_path: str, rank: int) -> None:
    if rank == 0:
        save_json(results, output_path)
        print(f"\nResults saved to: {output_path}")
