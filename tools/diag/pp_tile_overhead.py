"""Per-tile fixed cost of the 256² ping-pong NT GEMM (diagnostic).

One round of tiles (M = N = 4096: 256 tiles on 256 CUs) at K = 256 .. 8192, the balanced
ping-pong forced (``set_stagger(7)``). From per-workgroup stamps (``utils.stamps``) the median
workgroup time is fitted as ``a + b * nk`` (nk = K / 64 K-tiles): ``a`` is what every tile pays
besides its K-loop (prologue loads, pipeline fill / drain, epilogue stores) — the most a persistent,
cross-tile-pipelined schedule could recover per tile. Also prints the kernel time (events) per K.
"""

from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    import torch

    from distributed_llm_backend_benchmark_amd.ops import gemm, linear
    from distributed_llm_backend_benchmark_amd.utils.stamps import Stamps, summarize

    os.environ["DLBB_GEMM"] = "mfma"
    gemm.set_tile(256)
    gemm.set_stagger(7)
    dev = torch.device("cuda", 0)
    M = N = int(os.environ.get("PP_MN", "4096"))
    pts = []
    for K in (256, 512, 1024, 2048, 4096, 8192):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for _ in range(5):
            linear(x, w, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            linear(x, w, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        meds = []
        for _ in range(3):
            with Stamps(1 << 16) as st:
                linear(x, w, out=out)
            s = summarize(st.collect())
            meds.append(s[0]["median_wg_ns"] / 1e3)
        med = sorted(meds)[1]
        nk = K // 64
        pts.append((nk, med))
        print(json.dumps({"M": M, "N": N, "K": K, "nk": nk, "kernel_us": round(us, 2),
                          "median_wg_us": round(med, 2),
                          "tflops": round(2 * M * N * K / us / 1e6, 1)}), flush=True)
    n = len(pts)
    sx = sum(p[0] for p in pts)
    sy = sum(p[1] for p in pts)
    sxx = sum(p[0] ** 2 for p in pts)
    sxy = sum(p[0] * p[1] for p in pts)
    b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
    a = (sy - b * sx) / n
    print(json.dumps({"fit": "median_wg_us = a + b * nk", "a_us": round(a, 3),
                      "b_us_per_ktile": round(b, 4),
                      "overhead_at_nk64_pct": round(100 * a / (a + 64 * b), 2),
                      "overhead_at_nk12_pct": round(100 * a / (a + 12 * b), 2)}), flush=True)


if __name__ == "__main__":
    main()
