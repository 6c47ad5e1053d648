"""A/B of the attention backward with incremental DMA sources (dlbb_attn_set_bwd_incr bit mask:
1 dQ kernel, 2 dK/dV kernel) at the GPT-2 shape and two longer ones; interleaved rounds,
best-of. One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd  # noqa: E402

lib = _lib.lib()
MODES = (0, 1, 2, 3)
for B, T, H in ((16, 1024, 12), (8, 2048, 12), (4, 4096, 16)):
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    go = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
    o, lse = attn_fwd(qkv, H)
    best = {m: 1e9 for m in MODES}
    for _ in range(6):
        for m in MODES:
            lib.dlbb_attn_set_bwd_incr(m)
            attn_bwd(qkv, o, lse, go, H)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                attn_bwd(qkv, o, lse, go, H)
            e.record()
            e.synchronize()
            best[m] = min(best[m], s.elapsed_time(e) / 10 * 1e3)
    lib.dlbb_attn_set_bwd_incr(1)
    print(json.dumps({"B": B, "T": T, "H": H, "bwd_us": {m: round(t, 2) for m, t in best.items()}}),
          flush=True)
