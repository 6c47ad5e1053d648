"""A/B the attention kernels' XCD-aware head-contiguous block order, interleaved in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd  # noqa: E402
from wgrad_ab import timed  # noqa: E402

for B, T, H in ((16, 1024, 12), (8, 2048, 12), (4, 4096, 16), (1, 8192, 16)):
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    go = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
    res = {}
    outs = {}
    for _ in range(5):
        for on in (0, 1):
            _lib.lib().dlbb_attn_set_xcd(on)
            o, lse = attn_fwd(qkv, H)
            tf = timed(lambda: attn_fwd(qkv, H))
            tb = timed(lambda: attn_bwd(qkv, o, lse, go, H), iters=10)
            r = res.setdefault(on, [1e9, 1e9])
            r[0], r[1] = min(r[0], tf), min(r[1], tb)
            outs[on] = (o.float(), attn_bwd(qkv, o, lse, go, H).float())
    _lib.lib().dlbb_attn_set_xcd(1)
    same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    fl = 4.0 * B * H * T * T * 64 / 2
    print(json.dumps({"B": B, "T": T, "H": H,
                      "fwd_us": {k: round(v[0] * 1e6, 1) for k, v in res.items()},
                      "bwd_us": {k: round(v[1] * 1e6, 1) for k, v in res.items()},
                      "fwd_tflops_xcd": round(fl / res[1][0] / 1e12, 1),
                      "bwd_tflops_xcd": round(2.5 * fl / res[1][1] / 1e12, 1),
                      "bitwise_same": same}), flush=True)
