"""Every GEMM of one GPT-2-small training step (B16 x T1024 = 16384 tokens), ours vs the library,
device time (best of 5 rounds x 20 iterations, HIP events), TFLOP/s. One JSON line per GEMM.

fwd   : y = act(x W^T + b)      ours = fused MFMA kernel          lib = hipBLASLt addmm + our epilogue
dgrad : dX = dY W               ours = MFMA NT kernel on W^T copy  lib = hipBLASLt
wgrad : dW = dY^T X (+ db)      ours = split-K TN kernel           lib = hipBLASLt (+ torch colsum)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm as G  # noqa: E402


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


def main():
    M, C, V = 16384, 768, 50304
    layers = [("qkv", 3 * C, C, None, True), ("proj", C, C, None, True),
              ("fc", 4 * C, C, "gelu_tanh", True), ("mproj", C, 4 * C, None, True),
              ("lmhead", V, C, None, False)]
    dev = "cuda"
    for name, N, K, act, has_b in layers:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        b = (torch.rand(N, device=dev) * 0.1).to(torch.bfloat16) if has_b else None
        dy = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if act else None
        fl = 2.0 * M * N * K
        args = (x, w, b, act, None, out, pre)
        f_ours = t_best(lambda: G._mfma_linear(*args))
        f_lib = t_best(lambda: G._blas_linear(*args))
        wt = w.t().contiguous()
        d_lib = t_best(lambda: torch.matmul(dy, w))
        d_ours = t_best(lambda: G._mfma_linear(dy, wt, None, None, None,
                                               torch.empty(M, K, device=dev,
                                                           dtype=torch.bfloat16), None))
        t_tr = t_best(lambda: w.t().contiguous())
        dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        db = torch.empty(N, device=dev, dtype=torch.bfloat16) if has_b else None
        g_ours = t_best(lambda: G._wgrad_hip(dy, x, dw, False, None, db))
        g_lib = t_best(lambda: G._wgrad_blas(dy, x, dw, False, None, db))
        tf = lambda t: round(fl / t / 1e12, 1)  # noqa: E731
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K,
                          "fwd_us": [round(f_ours * 1e6, 1), round(f_lib * 1e6, 1)],
                          "fwd_tflops": [tf(f_ours), tf(f_lib)],
                          "dgrad_us": [round(d_ours * 1e6, 1), round(d_lib * 1e6, 1)],
                          "dgrad_tflops": [tf(d_ours), tf(d_lib)],
                          "transpose_us": round(t_tr * 1e6, 1),
                          "wgrad_us": [round(g_ours * 1e6, 1), round(g_lib * 1e6, 1)],
                          "wgrad_tflops": [tf(g_ours), tf(g_lib)],
                          "order": "[ours, library]"}), flush=True)


if __name__ == "__main__":
    main()
