"""Deterministic fault injection for the sweep engine's failure handling.

The reference swallows per-config failures with ``try/except … continue``
(``collectives/1d/openmpi.py:254-267``, ``collectives/1d/dsccl.py:207-223``), so a failed
config silently has no output. Our sweeps agree on setup failure across ranks and
write ``<stem>.error.json``; this module lets tests (and operators) trigger exactly that path:

    DLBB_FAULT_INJECT="op=allreduce,size=1KB,rank=1,stage=setup"

fails the setup of the ``allreduce`` / ``1KB`` config on rank 1 (``stage=run`` raises after the
setup agreement instead, on every rank, to exercise the per-config error record;
``stage=corrupt`` perturbs the op's RESULT on ``rank`` after the validation run — a collective
that silently returned wrong data — to exercise the ``wrong_result`` refusal). Keys are
optional; an empty spec injects nothing. ``size`` matches the 1D size label or the 3D shape
string ``b<B>_s<S>_h<H>``.
"""

from __future__ import annotations

import os
from typing import Dict, Optional


class InjectedFault(RuntimeError):
    pass


def _spec() -> Dict[str, str]:
    raw = os.environ.get("DLBB_FAULT_INJECT", "").strip()
    if not raw:
        return {}
    out = {}
    for part in raw.split(","):
        k, _, v = part.partition("=")
        if k.strip():
            out[k.strip()] = v.strip()
    return out


def maybe_fail(stage: str, op: str, size: str, rank: int) -> None:
    spec = _spec()
    if not spec:
        return
    if spec.get("stage", "setup") != stage:
        return
    if "op" in spec and spec["op"] != op:
        return
    if "size" in spec and spec["size"] != size:
        return
    if "rank" in spec and stage == "setup" and int(spec["rank"]) != rank:
        return
    raise InjectedFault(f"injected fault ({stage}) op={op} size={size} rank={rank}")


def maybe_corrupt(op: str, size: str, rank: int, result) -> bool:
    """``stage=corrupt``: add 1 to the first element of ``result`` (a tensor) on the matching
    rank; returns whether it did."""
    spec = _spec()
    if not spec or spec.get("stage") != "corrupt":
        return False
    if "op" in spec and spec["op"] != op:
        return False
    if "size" in spec and spec["size"] != size:
        return False
    if "rank" in spec and int(spec["rank"]) != rank:
        return False
    if result is None or result.numel() == 0:
        return False
    flat = result.reshape(-1)
    flat[:1] += 1
    return True


def active() -> Optional[Dict[str, str]]:
    return _spec() or None
