"""A/B the NN (dgrad) MFMA kernel against hipBLASLt on the backward input-gradient shapes of
GPT-2 and the TP 7B model, in ONE process, interleaved rounds, random operands. One JSON line
per shape: dX[M, N] = dY[M, K] @ W[K, N] (W = the Linear weight [out, in]).

    python tools/dgrad_ab.py [--rounds 5] [--iters 10] [--shapes gpt2_qkv,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm  # noqa: E402

# (name, M tokens, N = in_features (output of dgrad), K = out_features (reduction))
SHAPES = [("gpt2_qkv", 16384, 768, 2304), ("gpt2_attnproj", 16384, 768, 768),
          ("gpt2_fc", 16384, 768, 3072), ("gpt2_fcproj", 16384, 3072, 768),
          ("gpt2_lmhead", 16384, 768, 50304), ("7B_qkv_P1", 4096, 4096, 12288),
          ("7B_up_P1", 4096, 4096, 16384), ("7B_down_P1", 4096, 16384, 4096),
          ("sq8192", 8192, 8192, 8192)]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e-3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default=None)
    args = ap.parse_args()
    shapes = [s for s in SHAPES if not args.shapes or s[0] in args.shapes.split(",")]
    for name, M, N, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        dy = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(K, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = torch.matmul(dy.float(), w.float())
        gemm._dgrad_hip(dy, w, out)
        err = float((out.float() - ref).abs().max() / ref.abs().max())
        t_ours = t_blas = 1e9
        t_bal = {0: 1e9, 1: 1e9}
        for _ in range(args.rounds):
            for bal in (0, 1):
                gemm.set_bal(bal)
                t_bal[bal] = min(t_bal[bal], timed(lambda: gemm._dgrad_hip(dy, w, out),
                                                   args.iters))
            gemm.set_bal(2)
            t_ours = min(t_ours, timed(lambda: gemm._dgrad_hip(dy, w, out), args.iters))
            t_blas = min(t_blas, timed(lambda: torch.matmul(dy, w, out=out), args.iters))
        fl = 2.0 * M * N * K
        print(json.dumps({"case": name, "M": M, "N": N, "K": K,
                          "nn_ms": round(t_ours * 1e3, 4), "blas_ms": round(t_blas * 1e3, 4),
                          "nn_plain_ms": round(t_bal[0] * 1e3, 4),
                          "nn_bal_ms": round(t_bal[1] * 1e3, 4),
                          "nn_tflops": round(fl / t_ours / 1e12, 1),
                          "hipblaslt_tflops": round(fl / t_blas / 1e12, 1),
                          "rel_err_vs_fp32": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
