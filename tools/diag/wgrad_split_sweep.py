"""Diagnostic: the GPT-2 weight-gradient shapes (dW = dY^T X over 16384 tokens, fused bias
gradient) on each 128-class wgrad tile with split-K factors around the library heuristic —
device time per call (best of 5 x 10). One JSON line per (shape, tile, split)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_backend_benchmark_amd.ops import gemm  # noqa: E402


def timed(fn, iters=10, rounds=5):
    best = 1e9
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


M, C = 16384, 768
g = torch.Generator(device="cuda").manual_seed(0)
for name, N, K in (("qkv", 3 * C, C), ("proj", C, C), ("fc", 4 * C, C), ("mproj", C, 4 * C)):
    dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    db = torch.empty(N, device="cuda", dtype=torch.bfloat16)
    for tile, bn, bk in (("mfma", 128, 128), ("mfma256", 256, 128), ("mfma_wide", 128, 256)):
        if (bn == 256 and N % 256) or (bk == 256 and K % 256):
            continue
        tiles = (N // bn) * (K // bk)
        base = max(1, min(M // 256, (-(-768 // tiles)) if bn == bk == 128 else max(1, 512 // tiles)))
        for sp in sorted({max(1, base // 2), max(1, (base * 3) // 4), base, base + 1,
                          (base * 3) // 2, base * 2}):
            if sp > M // 256:
                continue
            ms = timed(lambda: gemm._wgrad_hip(dy, x, out, False, sp, db, bn=bn, bk=bk))
            print(json.dumps({"shape": name, "N": N, "K": K, "tile": tile, "tiles": tiles,
                              "split": sp, "heuristic": sp == base, "ms": round(ms, 4)}),
                  flush=True)
