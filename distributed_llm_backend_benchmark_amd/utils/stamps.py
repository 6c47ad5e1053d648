"""Per-workgroup start / end stamps of selected kernels (diagnostic).

``with Stamps(capacity) as st: ...; recs = st.collect()`` makes every launch of the stamped
kernels inside the block (the six ping-pong GEMMs, the n-way reduction, the spin stand-in)
run its stamped twin, which writes one record per workgroup: start and end time
(``s_memrealtime``, 100 MHz, one clock for the whole chip), the CU / SIMD / shader-engine ids
(``HW_REG_HW_ID``) and the XCD (``HW_REG_XCC_ID``). A store of 32 bytes per workgroup does not
serialise dispatch the way a profiler's kernel trace does, so contention between concurrent
grids (e.g. a comm stream beside the backward pass) stays visible.
"""

from __future__ import annotations

import ctypes
from typing import Dict, List

import torch

from ..ops import _lib

KINDS = {1: "gemm_nt_pp", 2: "gemm_nn_pp", 3: "gemm_tn_pp", 4: "reduce_sum", 5: "spin"}
TICK_NS = 10.0          # s_memrealtime runs at 100 MHz


def decode_hw_id(hw: int) -> Dict[str, int]:
    """gfx9 HW_ID fields: wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13."""
    return {"wave": hw & 15, "simd": (hw >> 4) & 3, "cu": (hw >> 8) & 15, "sh": (hw >> 12) & 1,
            "se": (hw >> 13) & 7}


class Stamps:
    def __init__(self, capacity_records: int = 1 << 20, device=None):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.buf = torch.zeros(capacity_records * 4, dtype=torch.int64, device=self.device)
        self.capacity = capacity_records

    def __enter__(self):
        torch.cuda.synchronize(self.device)
        _lib.lib().dlbb_stamps_set(self.buf.data_ptr(), self.capacity)
        return self

    def __exit__(self, *exc):
        torch.cuda.synchronize(self.device)
        self._entries = self._read_log()
        _lib.lib().dlbb_stamps_set(None, 0)
        return False

    def _read_log(self):
        lib = _lib.lib()
        n = int(lib.dlbb_stamps_launches())
        out = []
        kind, first, count = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64()
        for i in range(n):
            _lib.check(lib.dlbb_stamps_entry(i, ctypes.byref(kind), ctypes.byref(first),
                                             ctypes.byref(count)), "stamps_entry")
            out.append((int(kind.value), int(first.value), int(count.value)))
        return out

    def collect(self) -> List[dict]:
        """One dict per stamped launch, in launch order: kind, workgroup count and per-workgroup
        arrays (``start_ns``, ``end_ns`` relative to the first stamp of the whole collection,
        ``xcc``, ``cu``, ``se``)."""
        recs = self.buf.view(-1, 4).cpu()
        used = [e for e in self._entries]
        if not used:
            return []
        t_min = min(int(recs[f:f + c, 0].min()) for _, f, c in used)
        out = []
        for i, (kind, f, c) in enumerate(used):
            r = recs[f:f + c]
            hw = r[:, 2] & 0xFFFFFFFF
            out.append({
                "launch": i, "kind": KINDS.get(kind, str(kind)), "workgroups": c,
                "start_ns": ((r[:, 0] - t_min).double() * TICK_NS).tolist(),
                "end_ns": ((r[:, 1] - t_min).double() * TICK_NS).tolist(),
                "xcc": (r[:, 2] >> 32).tolist(),
                "cu": ((hw >> 8) & 15).tolist(),
                "se": ((hw >> 13) & 7).tolist(),
            })
        return out


def summarize(launches: List[dict]) -> List[dict]:
    """Per launch: first start, last start (dispatch spread), last end, median workgroup
    duration (ns)."""
    out = []
    for L in launches:
        s, e = L["start_ns"], L["end_ns"]
        d = sorted(b - a for a, b in zip(s, e))
        out.append({"launch": L["launch"], "kind": L["kind"], "workgroups": L["workgroups"],
                    "first_start_ns": min(s), "last_start_ns": max(s), "last_end_ns": max(e),
                    "dispatch_spread_ns": max(s) - min(s),
                    "median_wg_ns": d[len(d) // 2], "max_wg_ns": d[-1]})
    return out
