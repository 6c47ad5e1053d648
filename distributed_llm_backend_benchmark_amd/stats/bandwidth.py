"""Bandwidth conventions.

Two conventions are reported side by side:

* ``legacy_bandwidth_gbps`` — the reference's own column, ``N·2·P / max_time / 2^30`` for
  EVERY op with the element size hard-wired to 2 bytes (reference ``collectives/1d/stats.py:77-129``).
  Kept bit-compatible so our CSVs line up with the committed reference CSVs.
* ``algbw`` / ``busbw`` (GB/s, 1e9) — nccl-tests conventions, from the true byte count.
  ``bytes`` is the per-rank *message* size as the sweep defines it (the input tensor of one rank):

  ============== ====================================== ===========================
  op             algbw                                  busbw factor
  ============== ====================================== ===========================
  allreduce      bytes / t                              2(P-1)/P
  allgather      P*bytes / t  (output size)             (P-1)/P
  reduce_scatter bytes / t    (input size)              (P-1)/P
  alltoall       bytes / t    (send buffer)             (P-1)/P
  alltoall_moe   bytes / t    (send buffer, uneven)     (P-1)/P
  gather         P*bytes / t  (root receive buffer)     (P-1)/P
  scatter        P*bytes / t  (root send buffer)        (P-1)/P
  broadcast      bytes / t                              1
  reduce         bytes / t                              1
  sendrecv       bytes / t                              1
  ============== ====================================== ===========================

At P = 1 every factor with (P-1) is 0: there is no inter-GPU traffic, busBW is 0 by definition.
"""

from __future__ import annotations

from typing import Optional

GB = 1e9
GIB = float(1024 ** 3)

_OUTPUT_SCALED = {"allgather", "gather", "scatter"}
_FACTOR = {
    "allreduce": lambda p: 2.0 * (p - 1) / p,
    "allgather": lambda p: (p - 1) / p,
    "reduce_scatter": lambda p: (p - 1) / p,
    "alltoall": lambda p: (p - 1) / p,
    "alltoall_moe": lambda p: (p - 1) / p,
    "gather": lambda p: (p - 1) / p,
    "scatter": lambda p: (p - 1) / p,
    "broadcast": lambda p: 1.0,
    "reduce": lambda p: 1.0,
    "sendrecv": lambda p: 1.0,
}

KNOWN_OPS = tuple(_FACTOR.keys())


def bus_factor(op: str, num_ranks: int) -> float:
    if op not in _FACTOR:
        raise KeyError(f"unknown op {op!r}")
    return _FACTOR[op](int(num_ranks))


def algbw_gbps(op: str, nbytes: float, seconds: float, num_ranks: int) -> Optional[float]:
    if seconds is None or seconds <= 0:
        return None
    scale = num_ranks if op in _OUTPUT_SCALED else 1
    return (nbytes * scale / seconds) / GB


def busbw_gbps(op: str, nbytes: float, seconds: float, num_ranks: int) -> Optional[float]:
    a = algbw_gbps(op, nbytes, seconds, num_ranks)
    if a is None:
        return None
    return a * bus_factor(op, num_ranks)


def legacy_bandwidth_gbps(num_elements: int, seconds: float, num_ranks: int,
                          op: str = "allreduce") -> Optional[float]:
    """Reference ``collectives/1d/stats.py:77-129``: identical volume for every op,
    element size fixed at 2 B, GiB/s."""
    if op not in _FACTOR:
        return None
    if seconds is None or seconds <= 0:
        return None
    return (num_elements * 2 * num_ranks / seconds) / GIB


# ------------------------------------------------------------------------------ rooflines
# Ceilings a real measurement cannot beat (bench.py refuses a timing below them: such a call
# enqueued no work). Generous on purpose — they catch empty calls, not slow ones.
HBM_PEAK_GBPS = 8000.0            # MI355X HBM3E spec peak
ONDIE_PEAK_GBPS = 17200.0         # Infinity Cache / fabric ceiling for a working set on die
ONDIE_BYTES = 256 << 20           # Infinity Cache (MALL) capacity
XGMI_LINK_GBPS = 153.0            # one xGMI link (7 per GPU), taken per direction: generous

# minimum bytes the slowest rank's own memory reads + writes per call (message = ``nbytes`` per
# rank, as the sweep defines it); P = 1 collectives are timed out of place (a copy)
_LOCAL_TRAFFIC = {
    "allreduce": lambda b, p: 2.0 * b,                 # read input, write result
    "allgather": lambda b, p: (p + 1.0) * b,           # read own chunk, write P chunks
    "reduce_scatter": lambda b, p: b + b / p,
    "alltoall": lambda b, p: 2.0 * b,
    "alltoall_moe": lambda b, p: 2.0 * b,
    "gather": lambda b, p: (p + 1.0) * b,              # the root
    "scatter": lambda b, p: (p + 1.0) * b,
    "broadcast": lambda b, p: b,
    "reduce": lambda b, p: b,
    "sendrecv": lambda b, p: 2.0 * b,
}
# minimum bytes a rank must RECEIVE over its P - 1 links per call (any algorithm)
_RECV = {
    "allreduce": lambda b, p: b * (p - 1) / p,
    "allgather": lambda b, p: b * (p - 1.0),
    "reduce_scatter": lambda b, p: b * (p - 1) / p,
    "alltoall": lambda b, p: b * (p - 1) / p,
    "alltoall_moe": lambda b, p: b * (p - 1) / p,
    "broadcast": lambda b, p: b,
    "sendrecv": lambda b, p: b,
}


def min_seconds(op: str, nbytes: float, num_ranks: int, colocated: bool = False) -> float:
    """Lower bound on one call's time: the rank's own memory traffic at the HBM peak (the on-die
    cache ceiling when it fits in the 256 MiB Infinity Cache) and, at P > 1, the bytes it must
    receive spread over all P - 1 xGMI links at the link peak. ``colocated``: all P ranks share
    ONE device (rehearsals on a one-GPU box) — no link is crossed and the bound is the P ranks'
    combined local traffic on that device's memory."""
    p = int(num_ranks)
    if op not in _LOCAL_TRAFFIC:
        raise KeyError(f"unknown op {op!r}")
    local = _LOCAL_TRAFFIC[op](float(nbytes), p)
    if colocated and p > 1:
        local *= p
        peak = ONDIE_PEAK_GBPS if local <= ONDIE_BYTES else HBM_PEAK_GBPS
        return local / (peak * GB)
    peak = ONDIE_PEAK_GBPS if local <= ONDIE_BYTES else HBM_PEAK_GBPS
    t = local / (peak * GB)
    if p > 1 and op in _RECV:
        t = max(t, _RECV[op](float(nbytes), p) / ((p - 1) * XGMI_LINK_GBPS * GB))
    return t


def roofline_violation(op: str, nbytes: float, seconds: float, num_ranks: int,
                       colocated: bool = False) -> Optional[str]:
    """None when ``seconds`` is physically possible for ``op``; else the reason (an empty call
    or a timing that missed the work) — never report such a number."""
    if seconds is None or seconds <= 0:
        return "non-positive time"
    floor = min_seconds(op, nbytes, num_ranks, colocated)
    if seconds < floor:
        return (f"{op} of {int(nbytes)} B at P={num_ranks}"
                f"{' (ranks on one device)' if colocated else ''} took {seconds * 1e6:.3f} us, "
                f"below the {floor * 1e6:.3f} us memory/link roofline")
    return None

