"""LM-head forward (16384 x 50304 x 768, NT) under the GEMM schedule knobs: 256^2 ping-pong
(plain / balanced), deep 256^2 (mode 3), persistent 256^2 (mode 4), 128^2 tiles; vs hipBLASLt."""
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
    return s.elapsed_time(e) / iters


def main():
    M, N, K = 16384, 50304, 768
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = torch.matmul(x[:512].float(), w.float().t())

    def ours(tile, stagger, bal):
        def run():
            G.set_tile(tile)
            G.set_stagger(stagger)
            G.set_bal(bal)
            G._mfma_linear(x, w, None, None, None, out, None)
        return run
    impls = {"pp_plain": ours(0, 6, 0), "pp_bal": ours(0, 6, 1), "deep": ours(256, 3, 2),
             "persistent": ours(256, 4, 2), "t128": ours(128, 6, 2),
             "blas": lambda: torch.matmul(x, w.t(), out=out)}
    best, err = {k: 1e9 for k in impls}, {}
    for _ in range(5):
        for k, fn in impls.items():
            best[k] = min(best[k], timed(fn))
            err[k] = float((out[:512].float() - ref).abs().max() / ref.abs().max())
    G.set_tile(0)
    G.set_stagger(6)
    G.set_bal(2)
    print(json.dumps({"shape": [M, N, K], "ms": {k: round(v, 4) for k, v in best.items()},
                      "tflops": {k: round(2 * M * N * K / v / 1e9, 1) for k, v in best.items()},
                      "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
