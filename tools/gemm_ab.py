"""A/B the 256^2 MFMA GEMM schedules (and hipBLASLt) in ONE process, interleaved rounds, random
operands (CDNA guide §5.4: zero-filled operands read high). Prints one JSON line per shape.

    python tools/gemm_ab.py [--modes 1,3] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd import ops  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.gemm import set_stagger, set_tile  # noqa: E402

SHAPES = [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
          ("7B_qkv_P1", 4096, 12288, 4096), ("7B_up_P1", 4096, 16384, 4096),
          ("7B_down_P1", 4096, 4096, 16384), ("gpt2_lmhead", 16384, 50304, 768),
          ("gpt2_fc", 16384, 3072, 768), ("7B_qkv_P8", 4096, 1536, 4096),
          ("7B_up_P8", 4096, 2048, 4096), ("7B_down_P8", 4096, 4096, 2048),
          ("1B_qkv_P8", 1024, 768, 2048)]


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
    ap.add_argument("--modes", default="1,3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--tile", type=int, default=256, help="force the 128^2 or 256^2 kernel")
    args = ap.parse_args()
    modes = [int(m) for m in args.modes.split(",")]
    os.environ["DLBB_GEMM"] = "mfma"
    set_tile(args.tile)
    shapes = [s for s in SHAPES if not args.shapes or s[0] in args.shapes.split(",")]
    for name, M, N, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        ref = torch.matmul(x, w.t())
        errs = {}
        for m in modes:
            set_stagger(m)
            y = ops.linear(x, w)
            errs[m] = float((y.float() - ref.float()).abs().max())
        best = {m: 1e9 for m in modes}
        best_blas = 1e9
        for _ in range(args.rounds):
            for m in modes:
                set_stagger(m)
                best[m] = min(best[m], timed(lambda: ops.linear(x, w), args.iters))
            best_blas = min(best_blas, timed(lambda: torch.matmul(x, w.t()), args.iters))
        fl = 2.0 * M * N * K
        print(json.dumps({"case": name, "M": M, "N": N, "K": K,
                          **{f"mode{m}_tflops": round(fl / best[m] / 1e12, 1) for m in modes},
                          "hipblaslt_tflops": round(fl / best_blas / 1e12, 1),
                          "max_abs_err_vs_blas": errs}), flush=True)
    set_tile(0)


if __name__ == "__main__":
    main()
