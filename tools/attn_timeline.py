"""Per-workgroup timeline of the attention kernels (wg_stamp in csrc/attention.hip): the 100 MHz
wall clock at each workgroup's start, at the end of its first causal pass and at its end, plus the
CU it ran on. Reports kernel span, workgroup duration spread, start-time spread (dispatch ramp /
later rounds) and how many workgroups each CU held at once — the residency that the PMC
estimate (SQ_WAVE_CYCLES x 4 / kernel cycles) only gives as an average.

    python tools/attn_timeline.py [B T H] [--dump=DIR]   (default: the GPT-2 shape 16 1024 12,
    D = 64; --dump saves the last repetition's raw stamps as .npy)
"""
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd  # noqa: E402

TICK_US = 0.01   # wall_clock64: 100 MHz


def analyse(st: torch.Tensor, name: str, rec: dict):
    a = st.cpu().tolist()
    wg = [r for r in a if r[0] and r[2]]
    t0 = min(r[0] for r in wg)
    span = (max(r[2] for r in wg) - t0) * TICK_US
    dur = sorted((r[2] - r[0]) * TICK_US for r in wg)
    starts = sorted((r[0] - t0) * TICK_US for r in wg)
    p0 = sorted((r[1] - r[0]) * TICK_US for r in wg if r[1])
    per_cu = defaultdict(list)
    for r in wg:
        v = r[3]
        per_cu[(v >> 16, (v >> 5) & 7, (v >> 4) & 1, v & 15)].append((r[0], r[2]))
    peak = []
    for iv in per_cu.values():
        ev = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        peak.append(m)
    busy = sum(dur) / span          # mean workgroups resident over the span
    q = lambda v, f: round(v[min(len(v) - 1, int(f * len(v)))], 2)  # noqa: E731
    rec[name] = {"wgs": len(wg), "span_us": round(span, 2), "dur_us_min_med_max":
                 [q(dur, 0), q(dur, 0.5), q(dur, 1.0)],
                 "start_us_p50_p90_max": [q(starts, 0.5), q(starts, 0.9), q(starts, 1.0)],
                 "first_pass_us_med": q(p0, 0.5) if p0 else None,
                 "cus_used": len(per_cu), "wgs_per_cu_hist": _hist([len(v) for v in per_cu.values()]),
                 "peak_concurrent_per_cu_hist": _hist(peak),
                 "mean_resident_wgs": round(busy, 1),
                 "mean_resident_waves_per_simd": round(busy * 4 / 1024, 2)}


def _hist(v):
    h = defaultdict(int)
    for x in v:
        h[x] += 1
    return dict(sorted(h.items()))


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    xcd = next((int(x.split("=", 1)[1]) for x in sys.argv[1:] if x.startswith("--xcd=")), None)
    dump = next((x.split("=", 1)[1] for x in sys.argv[1:] if x.startswith("--dump=")), None)
    B, T, H = (int(x) for x in args[:3]) if len(args) >= 3 else (16, 1024, 12)
    D = 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, T, 3 * H * D, device="cuda", generator=g).to(torch.bfloat16)
    gout = torch.randn(B, T, H * D, device="cuda", generator=g).to(torch.bfloat16)
    nq = ((T + 127) // 128 + 1) // 2
    nk = ((T + 127) // 128 + 1) // 2   # dK/dV key blocks of 128 (kBwdKeys), paired
    sf = torch.zeros(nq * H * B, 4, dtype=torch.int64, device="cuda")
    sq = torch.zeros(nq * H * B, 4, dtype=torch.int64, device="cuda")
    sk = torch.zeros(nk * H * B * 2, 4, dtype=torch.int64, device="cuda")  # generous
    for _ in range(5):
        o, lse = attn_fwd(qkv, H)
        attn_bwd(qkv, o, lse, gout, H)
    torch.cuda.synchronize()
    L = _lib.lib()
    if xcd is not None:
        L.dlbb_attn_set_xcd(xcd)
    out = {"shape": [B, T, H, D]}
    for rep in range(3):
        sf.zero_(); sq.zero_(); sk.zero_()
        L.dlbb_attn_set_stamps(sf.data_ptr(), sq.data_ptr(), sk.data_ptr())
        o, lse = attn_fwd(qkv, H)
        attn_bwd(qkv, o, lse, gout, H)
        torch.cuda.synchronize()
        L.dlbb_attn_set_stamps(None, None, None)
        rec = {}
        analyse(sf, "fwd", rec)
        analyse(sq, "dq", rec)
        analyse(sk, "dkdv", rec)
        out[f"rep{rep}"] = rec
        if dump and rep == 2:
            import numpy as np
            os.makedirs(dump, exist_ok=True)
            for nm, t in (("fwd", sf), ("dq", sq), ("dkdv", sk)):
                np.save(os.path.join(dump, f"stamps_{nm}.npy"), t.cpu().numpy())
        print(json.dumps({"rep": rep, **rec}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
