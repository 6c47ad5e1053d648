"""A/B of the causal attention forward schedule variants (csrc/attention.hip
attn_fwd_d64_kernel<V>, bit mask: 1 batched K reads, 2 permlane32 max exchange, 4 incremental DMA
addresses) at the GPT-2 shape and two longer ones; rounds interleaved over variants, best-of
per variant. One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import attn_fwd  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("ATTN_VARIANTS", "0,2,4,6,7,14").split(",")]
lib = _lib.lib()
for B, T, H in ((16, 1024, 12), (8, 2048, 12), (4, 4096, 16)):
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    fl = 4.0 * B * H * T * T * 64 / 2
    best = {v: 1e9 for v in VARIANTS}
    ref = None
    err = {}
    for rnd in range(6):
        for v in VARIANTS:
            lib.dlbb_attn_set_fwd_variant(v)
            o, _ = attn_fwd(qkv, H)
            if rnd == 0:
                if ref is None:
                    ref = o.float()
                err[v] = float((o.float() - ref).abs().max())
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                attn_fwd(qkv, H)
            e.record()
            e.synchronize()
            best[v] = min(best[v], s.elapsed_time(e) / 20 * 1e3)
    lib.dlbb_attn_set_fwd_variant(0)
    print(json.dumps({"B": B, "T": T, "H": H,
                      "us": {v: round(t, 2) for v, t in best.items()},
                      "tflops": {v: round(fl / t / 1e6, 1) for v, t in best.items()},
                      "max_abs_diff_vs_v0": err}), flush=True)
