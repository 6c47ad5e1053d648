"""Forward GEMM on the GPT-2 shapes: 256^2 vs 128^2 MFMA kernel (fused epilogue) vs library,
interleaved rounds in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm as G  # noqa: E402
from wgrad_ab import timed  # noqa: E402


def main():
    M, C = 16384, 768
    for name, N, K, act in (("qkv", 3 * C, C, None), ("proj", C, C, None),
                            ("fc", 4 * C, C, "gelu_tanh"), ("fc_noact", 4 * C, C, None),
                            ("mproj", C, 4 * C, None)):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = (torch.rand(N, device="cuda") * 0.1).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if act else None
        args = (x, w, b, act, None, out, pre)
        res = {"t256": 1e9, "t128": 1e9, "lib": 1e9}
        for _ in range(5):
            G.set_tile(256)
            res["t256"] = min(res["t256"], timed(lambda: G._mfma_linear(*args)))
            G.set_tile(128)
            res["t128"] = min(res["t128"], timed(lambda: G._mfma_linear(*args)))
            G.set_tile(0)
            res["lib"] = min(res["lib"], timed(lambda: G._blas_linear(*args)))
        print(json.dumps({"gemm": name, "N": N, "K": K,
                          "us": {k: round(v * 1e6, 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
