"""Tiny driver for PMC-counter profiling: runs ONE op a few times (no timing logic).
usage: prof_target.py gemm256|gemm128|blas|reduce8|ln|xent"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd import ops  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.gemm import set_tile  # noqa: E402

what = sys.argv[1]
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
if what.startswith("gemm") or what == "blas":
    M = N = K = 8192
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    os.environ["DLBB_GEMM"] = "blas" if what == "blas" else "mfma"
    if what != "blas":
        set_tile(int(what[4:]))
    fn = lambda: ops.linear(x, w)  # noqa: E731
elif what == "reduce8":
    srcs = [torch.randn(1 << 25, device=dev, generator=g).to(torch.bfloat16) for _ in range(8)]
    fn = lambda: ops.reduce_sum(srcs)  # noqa: E731
elif what == "ln":
    x = torch.randn(4096, 8192, device=dev, generator=g).to(torch.bfloat16)
    r = torch.randn_like(x)
    wt = torch.ones(8192, device=dev, dtype=torch.bfloat16)
    fn = lambda: ops.layernorm(x, wt, wt, residual=r)  # noqa: E731
elif what == "xent":
    x = torch.randn(16384, 50304, device=dev, generator=g).to(torch.bfloat16)
    t = torch.randint(0, 50304, (16384,), device=dev)
    fn = lambda: ops.cross_entropy(x, t)  # noqa: E731
else:
    raise SystemExit(f"unknown target {what}")
for _ in range(5):
    fn()
torch.cuda.synchronize()
print("done", what)
