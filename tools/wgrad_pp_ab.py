"""A/B the 256^2 ping-pong weight-gradient kernel (TN, plain / balanced DMA issue, with and
without the split-K tail of a partial last round) against the
128^2 wgrad kernel (its own split heuristic) and hipBLASLt on the GPT-2 and 7B dW shapes
(no fused bias: the LM head; the others with a plain store as a kernel-only comparison).
Interleaved rounds in one process, best of 5; max relative error vs an fp32 product."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm as G  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e-3 / iters


def pp(bal, tail=True):
    def run(dy, x, dw):
        G.set_bal(bal)
        os.environ["DLBB_PP_TAIL"] = "1" if tail else "0"
        G._wgrad_pp(dy, x, dw, False)
        os.environ["DLBB_PP_TAIL"] = "1"
    return run


def main():
    C = 768
    impls = {"pp_plain": pp(0), "pp_bal": pp(1), "pp_bal_notail": pp(1, tail=False),
             "mfma128": lambda dy, x, dw: G._wgrad_hip(dy, x, dw, False),
             "blas": lambda dy, x, dw: G._wgrad_blas(dy, x, dw, False)}
    shapes = (("gpt2_lmhead", 16384, 50304, C), ("gpt2_fc", 16384, 4 * C, C),
              ("gpt2_mproj", 16384, C, 4 * C), ("gpt2_qkv", 16384, 3 * C, C),
              ("7b_qkv", 4096, 12288, 4096), ("7b_ffn_down", 4096, 4096, 16384),
              ("8192cube", 8192, 8192, 8192))
    for name, T, N, K in shapes:
        x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(T, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        ref = torch.matmul(dy.t().float(), x.float())
        best = {k: 1e9 for k in impls}
        errs = {}
        for _ in range(5):
            for k, fn in impls.items():
                if k.startswith("pp") and not G.wgrad_pp_supported(dy, x, dw, False):
                    continue
                best[k] = min(best[k], timed(lambda: fn(dy, x, dw)))
                errs[k] = float((dw.float() - ref).abs().max() / ref.abs().max())
        G.set_bal(2)
        fl = 2.0 * T * N * K
        best = {k: t for k, t in best.items() if t < 1e9}
        print(json.dumps({"gemm": name, "T": T, "N": N, "K": K,
                          "ms": {k: round(t * 1e3, 4) for k, t in best.items()},
                          "tflops": {k: round(fl / t / 1e12, 1) for k, t in best.items()},
                          "rel_err": errs}), flush=True)
        del x, dy, dw, ref


if __name__ == "__main__":
    main()
