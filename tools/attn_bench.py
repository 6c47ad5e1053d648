"""Device time of the causal attention forward / backward (ours vs torch SDPA vs the library
backward) at the GPT-2 shape and longer sequences, head dim 64 and 128."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import causal_attention  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import (  # noqa: E402
    _torch_attention, attn_bwd, attn_bwd_library, attn_fwd)


def t_best(fn, iters=20, rounds=5):
    best = 1e9
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e-3)
    return best


for B, T, H, D in ((16, 1024, 12, 64), (8, 2048, 12, 64), (4, 4096, 16, 64),
                   (16, 1024, 6, 128), (4, 4096, 8, 128)):
    qkv = torch.randn(B, T, 3 * H * D, device="cuda").to(torch.bfloat16)
    fl = 4.0 * B * H * T * T * D / 2          # causal
    t_ours = t_best(lambda: attn_fwd(qkv, H))
    t_torch = t_best(lambda: _torch_attention(qkv, H))
    x = qkv.clone().requires_grad_(True)
    go = torch.randn(B, T, H * D, device="cuda").to(torch.bfloat16)
    t_fb_ours = t_best(lambda: causal_attention(x, H).backward(go), iters=5, rounds=3)
    t_fb_torch = t_best(lambda: _torch_attention(x, H).backward(go), iters=5, rounds=3)
    o, lse = attn_fwd(qkv, H)
    rec = {"B": B, "T": T, "H": H, "D": D, "fwd_us_ours": t_ours * 1e6,
           "fwd_us_torch": t_torch * 1e6, "fwd_tflops_ours": fl / t_ours / 1e12,
           "fwd_tflops_torch": fl / t_torch / 1e12,
           "fwd_bwd_us_ours": t_fb_ours * 1e6, "fwd_bwd_us_torch": t_fb_torch * 1e6}
    t_lib = t_best(lambda: attn_bwd_library(qkv, o, lse, go, H), iters=10, rounds=3)
    rec["bwd_us_library"] = t_lib * 1e6
    if D == 64:
        t_bwd = t_best(lambda: attn_bwd(qkv, o, lse, go, H), iters=10, rounds=3)
        rec.update(bwd_us_ours=t_bwd * 1e6, bwd_tflops_ours=2.5 * fl / t_bwd / 1e12)
    print(json.dumps(rec), flush=True)
