"""Attention forward device time under the tree first on sys.path (A/B of two builds with
tools/ab_trees.sh-style PYTHONPATH switching): one JSON line, best of interleaved rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("PYTHONPATH", "").split(":")[0] or
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import attn_fwd  # noqa: E402

CASES = ((16, 1024, 12, 64), (8, 2048, 12, 64), (4, 4096, 16, 64), (16, 1024, 6, 128),
         (4, 4096, 8, 128))


def t_us(fn, iters=20):
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
for B, T, H, D in CASES:
    qkv = torch.randn(B, T, 3 * H * D, device="cuda", generator=g).to(torch.bfloat16)
    best = min(t_us(lambda: attn_fwd(qkv, H)) for _ in range(6))
    o, lse = attn_fwd(qkv, H)
    out[f"{B}x{T}x{H}x{D}"] = {"us": round(best, 2),
                               "digest": float(o.float().sum()) + float(lse.sum())}
print(json.dumps(out), flush=True)
