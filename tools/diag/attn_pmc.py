"""Run the causal attention kernels (forward, dQ, dK/dV) at the GPT-2 shape a fixed number of
times, for rocprofv3 PMC passes (one counter set per run):

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... --output-format csv -d OUT -- \
        python3 tools/diag/attn_pmc.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd  # noqa: E402

B, T, H = 16, 1024, 12
N = int(os.environ.get("ATTN_PMC_ITERS", "10"))
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(B, T, 3 * H * 64, device="cuda", generator=g).to(torch.bfloat16)
go = torch.randn(B, T, H * 64, device="cuda", generator=g).to(torch.bfloat16)
for _ in range(N):
    o, lse = attn_fwd(qkv, H)
for _ in range(N):
    attn_bwd(qkv, o, lse, go, H)
torch.cuda.synchronize()
print("ok", flush=True)
