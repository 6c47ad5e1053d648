"""Attention backward (dQ + dK/dV kernels, raw launcher) device time under the tree first on
sys.path, for an A/B of two builds: one JSON line, best of rounds, plus an output digest."""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("PYTHONPATH", "").split(":")[0] or
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd  # noqa: E402

CASES = ((16, 1024, 12), (8, 2048, 12), (4, 4096, 16))


def t_us(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


out = {"lib": _lib.LIB_PATH}
g = torch.Generator(device="cuda").manual_seed(0)
for B, T, H in CASES:
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda", generator=g).to(torch.bfloat16)
    go = torch.randn(B, T, H * 64, device="cuda", generator=g).to(torch.bfloat16)
    o, lse = attn_fwd(qkv, H)
    best = min(t_us(lambda: attn_bwd(qkv, o, lse, go, H)) for _ in range(5))
    d = attn_bwd(qkv, o, lse, go, H)
    out[f"{B}x{T}x{H}x64"] = {"us": round(best, 2), "digest": float(d.float().abs().sum())}
print(json.dumps(out), flush=True)
