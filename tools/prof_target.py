"""Tiny driver for PMC-counter profiling: runs ONE op a few times (no timing logic).
usage: prof_target.py longk|longkblas|attnfwd|attnbwd|lmhead|lmhead192|lmhead192p|lmheadblas|gemm256|gemm256s6|gemm256s7|gemm128|blas|nn|nnplain|tn|tnplain|wgrad128|
blastn|wgradqkv|wgradqkv256|reduce8|ln|xent|xentfused|embbwd"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd import ops  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.gemm import set_tile  # noqa: E402

what = sys.argv[1]
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
if what in ("attnfwd", "attnbwd"):   # causal attention at the GPT-2 step shape (B16 T1024 H12)
    from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd

    qkv = torch.randn(16, 1024, 3 * 12 * 64, device=dev, generator=g).to(torch.bfloat16)
    gout = torch.randn(16, 1024, 12 * 64, device=dev, generator=g).to(torch.bfloat16)
    o, lse = attn_fwd(qkv, 12)
    fn = ((lambda: attn_fwd(qkv, 12)) if what == "attnfwd"  # noqa: E731
          else (lambda: attn_bwd(qkv, o, lse, gout, 12)))
elif what.startswith("lmhead"):    # GPT-2 LM-head forward 16384 x 50304 x 768: lmhead (library
    # dispatch: 256² persistent), lmhead192 / lmhead192p (256 x 192 ping-pong / persistent spread
    # stores), lmheadblas (hipBLASLt)
    from distributed_llm_backend_benchmark_amd.ops import gemm as G

    x = torch.randn(16384, 768, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(50304, 768, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(16384, 50304, device=dev, dtype=torch.bfloat16)
    impl = {"lmhead": G._mfma_linear, "lmhead192": G._mfma192_linear,
            "lmhead192p": G._mfma192p_linear, "lmheadblas": G._blas_linear}[what]
    fn = lambda: impl(x, w, None, None, None, out, None)  # noqa: E731
elif what in ("longk", "longkblas"):   # single-round long-K NT GEMM 4096 x 4096 x 16384
    x = torch.randn(4096, 16384, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(4096, 16384, device=dev, generator=g).to(torch.bfloat16)
    os.environ["DLBB_GEMM"] = "blas" if what == "longkblas" else "mfma"
    fn = lambda: ops.linear(x, w)  # noqa: E731
elif what.startswith("gemm") or what == "blas":
    M = N = K = 8192
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    os.environ["DLBB_GEMM"] = "blas" if what == "blas" else "mfma"
    if what != "blas":             # gemm<tile>[s<schedule>], e.g. gemm256s6
        tile, _, sched = what[4:].partition("s")
        set_tile(int(tile))
        if sched:
            from distributed_llm_backend_benchmark_amd.ops.gemm import set_stagger

            set_stagger(int(sched))
    fn = lambda: ops.linear(x, w)  # noqa: E731
elif what in ("nn", "nnplain"):  # NN dgrad kernel (transposed-read W), balanced / plain DMA issue
    from distributed_llm_backend_benchmark_amd.ops import gemm as G

    M = N = K = 8192
    dy = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(K, N, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    G.set_bal(0 if what == "nnplain" else 1)
    fn = lambda: G._dgrad_hip(dy, w, out)  # noqa: E731
elif what in ("tn", "tnplain", "wgrad128", "blastn"):  # weight gradient dW = dY^T X at 8192^3
    from distributed_llm_backend_benchmark_amd.ops import gemm as G

    T = N = K = 8192
    dy = torch.randn(T, N, device=dev, generator=g).to(torch.bfloat16)
    xx = torch.randn(T, K, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    G.set_bal(0 if what == "tnplain" else 1)
    fn = {"tn": lambda: G._wgrad_pp(dy, xx, out, False),
          "tnplain": lambda: G._wgrad_pp(dy, xx, out, False),
          "wgrad128": lambda: G._wgrad_hip(dy, xx, out, False),
          "blastn": lambda: G._wgrad_blas(dy, xx, out, False)}[what]
elif what in ("wgradqkv", "wgradqkv256"):  # GPT-2 QKV dW 16384 x 2304 x 768 as in the step
    # (fused bias, bf16 accumulate): 128 x 256 tiles (wide, the step's choice) / 256 x 128
    from distributed_llm_backend_benchmark_amd.ops import gemm as G

    dy = torch.randn(16384, 2304, device=dev, generator=g).to(torch.bfloat16)
    xx = torch.randn(16384, 768, device=dev, generator=g).to(torch.bfloat16)
    out = torch.zeros(2304, 768, device=dev, dtype=torch.bfloat16)
    bo = torch.zeros(2304, device=dev, dtype=torch.bfloat16)
    impl = G._wgrad_hip_wide if what == "wgradqkv" else G._wgrad_hip256
    fn = lambda: impl(dy, xx, out, True, None, bo)  # noqa: E731
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
elif what == "xentfused":       # the in-place LM-head loss pass (v2), GPT-2 step shape
    from distributed_llm_backend_benchmark_amd.ops import _lib as L

    x = torch.randn(16384, 50304, device=dev, generator=g).to(torch.bfloat16)
    t = torch.randint(0, 50304, (16384,), device=dev)
    loss = torch.empty(16384, device=dev)
    sc = torch.full((1,), 1.0 / 16384, device=dev)
    fn = lambda: L.check(L.lib().dlbb_xent_fused(  # noqa: E731
        x.data_ptr(), t.data_ptr(), loss.data_ptr(), 16384, 50304, 50304, sc.data_ptr(),
        L.stream(x.device)), "xent_fused")
elif what == "embbwd":          # embedding backward into bf16 gradient buffers, GPT-2 shape
    from distributed_llm_backend_benchmark_amd.ops import _lib as L

    ids = torch.randint(0, 50304, (16384,), device=dev)
    s_ids, order = torch.sort(ids, stable=True)
    dx = torch.randn(16384, 768, device=dev, generator=g).to(torch.bfloat16)
    ge = torch.zeros(50304, 768, device=dev, dtype=torch.bfloat16)
    gp = torch.zeros(1024, 768, device=dev, dtype=torch.bfloat16)
    fn = lambda: L.check(L.lib().dlbb_embedding_bwd(  # noqa: E731
        s_ids.data_ptr(), order.data_ptr(), dx.data_ptr(), ge.data_ptr(), gp.data_ptr(),
        L.DT_BF16, 16384, 1024, 768, 50304, L.stream(dx.device)), "embedding_bwd")
else:
    raise SystemExit(f"unknown target {what}")
for _ in range(5):
    fn()
torch.cuda.synchronize()
print("done", what)
