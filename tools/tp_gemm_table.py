"""GEMM table of the TP transformer's per-rank shapes (reference models.py:47,81; shapes
models.py:126-144) at P = 1/2/4/8 plus the GPT-2 LM head: our dispatch vs hipBLASLt, one process,
interleaved rounds, uniform random operands (CDNA guide §5.4 rules 24/25). One JSON line per shape.

    python tools/tp_gemm_table.py [--model 7B] [--ps 1,2,4,8] [--rounds 5] [--modes auto]

``--modes``: comma list of our-kernel variants to time: ``auto`` = the library dispatch
(``DLBB_GEMM=mfma``), ``t128`` / ``t256`` force the tile, ``s<N>`` = set_stagger(N), ``v192`` =
the 256 x 192 tile variant (N % 192 == 0 shapes only), ``v192p`` / ``v192p18`` = its persistent
spread-store form (variant 2), ``sk`` = Stream-K on 256²
tiles (grids below one round of the CUs only), ``split`` = split-K ping-pong + reduce pass (same
grids). ``--gpt2`` adds the GPT-2 forward GEMMs.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd import ops  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops import _lib, gemm  # noqa: E402

CFG = {"1B": (2048, 8192), "7B": (4096, 16384), "13B": (5120, 20480)}


def tp_shapes(model: str, P: int, tokens: int):
    H, F = CFG[model]
    return [(f"{model}_qkv_P{P}", tokens, 3 * H // P, H),
            (f"{model}_out_P{P}", tokens, H, H // P),
            (f"{model}_up_P{P}", tokens, F // P, H),
            (f"{model}_down_P{P}", tokens, H, F // P)]


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


def set_mode(m):
    gemm.set_tile(0)
    gemm.set_stagger(6)
    if m == "t128":
        gemm.set_tile(128)
    elif m == "t256":
        gemm.set_tile(256)
    elif m.startswith("s") and m[1:].isdigit():
        gemm.set_stagger(int(m[1:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="7B")
    ap.add_argument("--ps", default="1,2,4,8")
    ap.add_argument("--tokens", type=int, default=4096, help="B*S (baseline 8 x 512)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default="auto")
    ap.add_argument("--lmhead", action="store_true", help="also the GPT-2 LM head forward")
    ap.add_argument("--gpt2", action="store_true",
                    help="also every GPT-2-small forward GEMM (B16 x T1024 = 16384 tokens)")
    ap.add_argument("--shapes", default=None, help="comma list of case names to keep")
    args = ap.parse_args()
    os.environ["DLBB_GEMM"] = "mfma"
    modes = args.modes.split(",")
    shapes = []
    for P in [int(p) for p in args.ps.split(",")]:
        shapes += tp_shapes(args.model, P, args.tokens)
    if args.lmhead or args.gpt2:
        shapes.append(("gpt2_lmhead", 16384, 50304, 768))
    if args.gpt2:
        shapes += [("gpt2_qkv", 16384, 2304, 768), ("gpt2_proj", 16384, 768, 768),
                   ("gpt2_fc", 16384, 3072, 768), ("gpt2_mproj", 16384, 768, 3072)]
    if args.shapes:
        keep = set(args.shapes.split(","))
        shapes = [s for s in shapes if s[0] in keep]
    for name, M, N, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        ref = (x.float() @ w.float().t())
        errs = {}
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ok = {"v192": gemm.mfma192_ok(M, N),
              "v192p": gemm.mfma192p_ok(M, N, K, True),
              "sk": gemm.streamk_ok(x, w),
              "split": gemm.split_plan(M, N, K, gemm._num_cus(x.device)) is not None}
        ms = [m for m in modes if ok.get(m, True)]

        def run(m):
            if m == "v192":      # 256 x 192 tiles (variant 1)
                return gemm._mfma192_linear(x, w, None, None, None, out, None)
            if m == "v192p":     # persistent, spread C stores (variant 2)
                return gemm._mfma192p_linear(x, w, None, None, None, out, None)
            if m == "sk":                 # Stream-K ping-pong, in-launch combine
                return gemm._mfma_streamk_linear(x, w, None, None, None, out, None)
            if m == "split":              # split-K ping-pong + reduce / cast pass
                return gemm._mfma_split_linear(x, w, None, None, None, out, None)
            return ops.linear(x, w)
        for m in ms:
            set_mode(m)
            y = run(m)
            errs[m] = float((y.float() - ref).abs().max() / ref.abs().max())
        best = {m: 1e9 for m in ms}
        best_blas = 1e9
        for _ in range(args.rounds):
            for m in ms:
                set_mode(m)
                best[m] = min(best[m], timed(lambda: run(m), args.iters))
            best_blas = min(best_blas, timed(lambda: torch.matmul(x, w.t()), args.iters))
        set_mode("auto")
        fl = 2.0 * M * N * K
        print(json.dumps({"case": name, "M": M, "N": N, "K": K,
                          **{f"{m}_ms": round(best[m] * 1e3, 4) for m in ms},
                          **{f"{m}_tflops": round(fl / best[m] / 1e12, 1) for m in ms},
                          "blas_ms": round(best_blas * 1e3, 4),
                          "blas_tflops": round(fl / best_blas / 1e12, 1),
                          "ours_vs_blas": round(best_blas / min(best.values()), 3),
                          "rel_err": errs}), flush=True)


if __name__ == "__main__":
    main()
