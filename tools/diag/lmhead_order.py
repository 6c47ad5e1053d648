"""Diagnostic: does the GPT-2 LM-head forward (16384 x 50304 x 768) depend on the order tiles are
handed out, and what do its C stores cost? Times our 256² persistent kernel (``mfma``) and the 256 x 192 spread-store persistent
kernel (``mfma192p``) for several GROUP_M values of ``tile_of`` (csrc/gemm.hip,
dlbb_gemm_set_group_m), against hipBLASLt. One JSON line per (kernel, group_m)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_backend_benchmark_amd.ops import _lib, gemm  # noqa: E402


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


M, N, K = 16384, 50304, 768
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
lib = _lib.lib()
print(json.dumps({"kernel": "blas", "ms": round(timed(lambda: torch.matmul(x, w.t())), 4)}),
      flush=True)
for name, fn in (("mfma", gemm._mfma_linear), ("mfma192p", gemm._mfma192p_linear)):
    for gm in (1, 2, 4, 8, 16, 32, 64):
        lib.dlbb_gemm_set_group_m(gm)
        ms = timed(lambda: fn(x, w, None, None, None, out, None))
        print(json.dumps({"kernel": name, "group_m": gm, "ms": round(ms, 4)}), flush=True)
lib.dlbb_gemm_set_group_m(0)
# the same kernels with their C stores compiled out: the K-loop's own time over the same tiles
lib.dlbb_gemm_set_diag_nostore(1)
for name, fn in (("mfma", gemm._mfma_linear), ("mfma192p", gemm._mfma192p_linear)):
    for gm in (1, 8):
        lib.dlbb_gemm_set_group_m(gm)
        ms = timed(lambda: fn(x, w, None, None, None, out, None))
        print(json.dumps({"kernel": name, "group_m": gm, "no_stores": True, "ms": round(ms, 4)}),
              flush=True)
lib.dlbb_gemm_set_diag_nostore(0)
lib.dlbb_gemm_set_group_m(0)
