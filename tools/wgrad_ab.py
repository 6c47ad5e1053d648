"""A/B the weight-gradient kernel's LDS ring depth (2/3/4 stages) on the GPT-2 dW shapes, fused
bias, interleaved rounds in one process; also checks each variant against the library."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm as G  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e-3 / iters


def main():
    M, C = 16384, 768
    stages = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,3,4").split(",")]
    for name, N, K in (("qkv", 3 * C, C), ("proj", C, C), ("fc", 4 * C, C), ("mproj", C, 4 * C),
                       ("lmhead", 50304, C)):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        bias = name != "lmhead"
        db = torch.empty(N, device="cuda", dtype=torch.bfloat16) if bias else None
        ref = torch.matmul(dy.t().float(), x.float())
        best = {nb: 1e9 for nb in stages}
        errs = {}
        for _ in range(5):
            for nb in stages:
                G.set_wgrad_stages(nb)
                best[nb] = min(best[nb], timed(lambda: G._wgrad_hip(dy, x, dw, False, None, db)))
                errs[nb] = float((dw.float() - ref).abs().max() / ref.abs().max())
        G.set_wgrad_stages(2)
        fl = 2.0 * M * N * K
        print(json.dumps({"gemm": name, "N": N, "K": K,
                          "us": {nb: round(t * 1e6, 1) for nb, t in best.items()},
                          "tflops": {nb: round(fl / t / 1e12, 1) for nb, t in best.items()},
                          "rel_err": errs}), flush=True)


if __name__ == "__main__":
    main()
