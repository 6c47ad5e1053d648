"""Diagnostic: the GPT-2 LM-head forward on each candidate kernel against an fp32 reference
(max |err| / max |ref|), on the step's shape and on realistic logits scale."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_backend_benchmark_amd.ops import gemm  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
M, N, K = 16384, 50304, 768
for scale in (0.02, 1.0):
    x = (torch.randn(M, K, device="cuda", generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * scale).to(torch.bfloat16)
    ref = x[:2048].float() @ w.float().t()
    for name, fn in (("mfma", gemm._mfma_linear), ("blas", gemm._blas_linear),
                     ("mfma192", gemm._mfma192_linear), ("mfma192p", gemm._mfma192p_linear)):
        out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        fn(x, w, None, None, None, out, None)
        torch.cuda.synchronize()
        err = (out[:2048].float() - ref).abs().max().item() / ref.abs().max().item()
        full_nan = bool(torch.isnan(out).any())
        # whole-matrix agreement with the library (every tile, not just the first rows)
        print(json.dumps({"scale": scale, "kernel": name, "rel_err_first2048": err,
                          "any_nan": full_nan}), flush=True)
        if name == "mfma":
            base = out.clone()
        else:
            d = (out.float() - base.float()).abs().max().item()
            print(json.dumps({"scale": scale, "kernel": name, "max_abs_diff_vs_mfma": d}),
                  flush=True)
