"""Where the GPT-2-small step's short-K / small-output GEMMs lose time (one process, device time,
best of rounds, uniform random operands).

wgrad : dW[N, K] = dY^T X (+ db) for the four per-layer linears (M = 16384 tokens):
        128^2 split-K kernel with the fused bias (today's choice) vs the 256^2 TN ping-pong with
        split-K s (no bias) + a column-sum pass for db
fwd   : y = x W^T (+ b, GELU): full epilogue vs plain output (plain is eligible for the
        persistent kernel) — the price of the epilogue on these shapes
dgrad : dX = dY W (NN) with and without the fused GELU backward

    python tools/diag/gpt2_small_gemm_probe.py > gpurun_out/gpt2_small_gemm_probe.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
    return round(best * 1e6, 1)


def main():
    M, C = 16384, 768
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)  # noqa
    for name, N, K in (("qkv", 3 * C, C), ("proj", C, C), ("fc", 4 * C, C), ("mproj", C, 4 * C)):
        dy, x = rnd(M, N), rnd(M, K)
        out = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        db = torch.empty(N, device=dev, dtype=torch.bfloat16)
        rec = {"gemm": name, "M": M, "N": N, "K": K}
        rec["wgrad128_bias_us"] = t_best(lambda: G._wgrad_hip(dy, x, out, False, None, db))
        if N % 256 == 0:
            rec["wgrad256x128_bias_us"] = t_best(lambda: G._wgrad_hip256(dy, x, out, False, None,
                                                                         db))
        rec["wgrad_wide_bias_us"] = t_best(lambda: G._wgrad_hip_wide(dy, x, out, False, None,
                                                                     db))
        for sw in (1, 2, 4, 8):
            rec[f"wgrad_wide_bias_s{sw}_us"] = t_best(
                lambda: G._wgrad_hip_wide(dy, x, out, False, sw, db))
        ref = (dy.float().t() @ x.float())
        pp = {}
        for s in (2, 3, 4, 6, 7, 8, 9, 12, 16, 28):
            tiles = (N // 256 if N % 256 == 0 else N // 128) * (K // 256)
            if s * tiles > 512 or s > M // 64:
                continue
            pp[s] = t_best(lambda: G._pp_launch(dy, x, out, False, 0, N, s))
        G._pp_launch(dy, x, out, False, 0, N, min(pp, key=pp.get))
        rec["pp_split_us"] = pp
        rec["pp_best_rel_err"] = float((out.float() - ref).abs().max() / ref.abs().max())
        rec["colsum_torch_us"] = t_best(lambda: dy.sum(0, dtype=torch.float32))
        # forward with the layer's epilogue vs plain
        xf, w, b = rnd(M, K), rnd(N, K), rnd(N)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        act = "gelu_tanh" if name == "fc" else None
        rec["fwd_epi_us"] = t_best(lambda: G._mfma_linear(xf, w, b, act, None, y,
                                                          pre if act else None))
        G.set_persist_epi(False)
        rec["fwd_epi_nopersist_us"] = t_best(lambda: G._mfma_linear(xf, w, b, act, None, y,
                                                                    pre if act else None))
        G.set_persist_epi(True)
        G.set_tile(128)
        rec["fwd_epi_t128_us"] = t_best(lambda: G._mfma_linear(xf, w, b, act, None, y,
                                                               pre if act else None))
        G.set_tile(0)
        rec["fwd_plain_us"] = t_best(lambda: G._mfma_linear(xf, w, None, None, None, y, None))
        rec["fwd_blas_epi_us"] = t_best(lambda: G._blas_linear(xf, w, b, act, None, y,
                                                               pre if act else None))
        print(json.dumps(rec), flush=True)
    # dgrad of the MLP proj through the GELU (NN kernel, EPI_DGELU) vs plain
    dy, w, u = rnd(M, C), rnd(C, 4 * C), rnd(M, 4 * C)
    dx = torch.empty(M, 4 * C, device=dev, dtype=torch.bfloat16)
    rec = {"gemm": "mproj_dgrad", "M": M, "N": 4 * C, "K": C,
           "dgrad_dgelu_us": t_best(lambda: G._dgrad_hip(dy, w, dx, None, (u, "gelu_tanh"))),
           "dgrad_plain_us": t_best(lambda: G._dgrad_hip(dy, w, dx, None, None)),
           "dgrad_dgelu_nopersist_us": None, "dgrad_plain_nopersist_us": None,
           "dgrad_blas_plain_us": t_best(lambda: G._dgrad_blas(dy, w, dx, None, None))}
    G.set_persist_epi(False)
    rec["dgrad_dgelu_nopersist_us"] = t_best(lambda: G._dgrad_hip(dy, w, dx, None,
                                                                  (u, "gelu_tanh")))
    rec["dgrad_plain_nopersist_us"] = t_best(lambda: G._dgrad_hip(dy, w, dx, None, None))
    G.set_persist_epi(True)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
