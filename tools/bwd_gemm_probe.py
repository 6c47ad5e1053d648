"""GPT-2 backward GEMM shapes: hipBLASLt (torch.matmul, the current backward) vs our NT MFMA
kernel on a transposed weight copy (dX = dY @ W == dY @ (W^T)^T) — device time, TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd import ops  # noqa: E402


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


M, C = 16384, 768
os.environ["DLBB_GEMM"] = "mfma"
for name, N_out, K_in in (("qkv", 3 * C, C), ("proj", C, C), ("fc", 4 * C, C), ("mproj", C, 4 * C)):
    w = (torch.randn(N_out, K_in, device="cuda") * 0.02).to(torch.bfloat16)   # [out, in]
    dy = torch.randn(M, N_out, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K_in, device="cuda").to(torch.bfloat16)
    fl = 2.0 * M * N_out * K_in
    t_dx_blas = t_best(lambda: torch.matmul(dy, w))
    wt = w.t().contiguous()                                                  # [in, out]
    t_tr = t_best(lambda: w.t().contiguous())
    ok = ops.gemm.hip_supported(dy, wt)
    t_dx_ours = t_best(lambda: ops.linear(dy, wt)) if ok else None
    err = float((ops.linear(dy, wt).float() - torch.matmul(dy, w).float()).abs().max()) if ok else None
    t_dw_blas = t_best(lambda: torch.matmul(dy.t(), x))
    from distributed_llm_backend_benchmark_amd.ops.gemm import wgrad
    t_dw_ours = t_best(lambda: wgrad(dy, x))
    dw_err = float((wgrad(dy, x).float() - torch.matmul(dy.t(), x).float()).abs().max())
    tiles = (N_out // 128) * (K_in // 128)
    splits = {}
    for target in (256, 512, 1024, 2048):
        sp = max(1, min(M // 256, -(-target // tiles)))
        splits[f"wgs{target}_split{sp}"] = round(t_best(lambda: wgrad(dy, x, split=sp)) * 1e6, 1)
    print(json.dumps({"gemm": name, "dX_shape": [M, K_in, N_out], "dX_blas_us": t_dx_blas * 1e6,
                      "dX_ours_us": None if t_dx_ours is None else t_dx_ours * 1e6,
                      "transpose_us": t_tr * 1e6, "dX_blas_tflops": fl / t_dx_blas / 1e12,
                      "dX_ours_tflops": None if t_dx_ours is None else fl / t_dx_ours / 1e12,
                      "dW_blas_us": t_dw_blas * 1e6, "dW_blas_tflops": fl / t_dw_blas / 1e12,
                      "dW_ours_us": t_dw_ours * 1e6, "dW_ours_tflops": fl / t_dw_ours / 1e12,
                      "dW_max_err": dw_err, "dW_ours_by_split_us": splits,
                      "max_err": err}), flush=True)
