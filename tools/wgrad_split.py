"""Sweep the weight-gradient kernel's split-K factor on the GPT-2 dW shapes (fused bias)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm as G  # noqa: E402
from wgrad_ab import timed  # noqa: E402


def main():
    M, C = 16384, 768
    for name, N, K in (("qkv", 3 * C, C), ("proj", C, C), ("fc", 4 * C, C), ("mproj", C, 4 * C),
                       ("lmhead", 50304, C)):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        db = torch.empty(N, device="cuda", dtype=torch.bfloat16) if name != "lmhead" else None
        tiles = (N // 128) * (K // 128)
        splits = sorted({max(1, min(M // 256, -(-t // tiles))) for t in (256, 384, 512, 768,
                                                                          1024, 1536)})
        best = {sp: 1e9 for sp in splits}
        for _ in range(4):
            for sp in splits:
                best[sp] = min(best[sp], timed(lambda: G._wgrad_hip(dy, x, dw, False, sp, db)))
        lib = min(timed(lambda: G._wgrad_blas(dy, x, dw, False, None, db)) for _ in range(3))
        fl = 2.0 * M * N * K
        print(json.dumps({"gemm": name, "tiles": tiles,
                          "us_by_split": {sp: round(t * 1e6, 1) for sp, t in best.items()},
                          "best_tflops": round(fl / min(best.values()) / 1e12, 1),
                          "lib_us": round(lib * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
