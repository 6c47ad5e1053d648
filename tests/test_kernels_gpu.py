"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference of the same op."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    from distributed_llm_backend_benchmark_amd.ops import _lib

    _lib.lib()  # must load: no silent fallback on a GPU box
    yield


def _randn(*shape, dtype=torch.bfloat16, seed=0, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("nsrc", [1, 2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize("n", [7, 4096, 1000003])
def test_reduce_sum(dtype, nsrc, n):
    from distributed_llm_backend_benchmark_amd.ops import reduce_sum

    srcs = [_randn(n, dtype=dtype, seed=i) for i in range(nsrc)]
    ref = sum(s.float() for s in srcs) * 0.5
    out = reduce_sum(srcs, out_dtype=torch.float32, scale=0.5)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    out2 = reduce_sum(srcs, scale=0.5)
    tol = 1e-2 if dtype != torch.float32 else 1e-5
    torch.testing.assert_close(out2.float(), ref, rtol=tol, atol=tol * nsrc)


@pytest.mark.parametrize("src,dst", [(torch.bfloat16, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.float16, torch.float32), (torch.float32, torch.float16),
                                     (torch.bfloat16, torch.float16)])
@pytest.mark.parametrize("n", [1, 13, 65536 + 5, 3 * 2048 * 256 + 3, 9 * 2048 * 256 * 8 + 1])
def test_cast(src, dst, n):
    """The cast (one 16-B wide side per lane, non-temporal stores) bit-exact against torch's
    conversion, with ragged tails, multi-tile grids past the 4096-block grid-stride cap, and an
    unaligned view (the one-element-per-lane kernel)."""
    from distributed_llm_backend_benchmark_amd.ops import cast

    x = _randn(n, dtype=src, seed=3)
    torch.testing.assert_close(cast(x, dst), x.to(dst), rtol=0, atol=0)
    if n > 1:
        torch.testing.assert_close(cast(x[1:], dst), x[1:].to(dst), rtol=0, atol=0)


def test_cast_nan_inf_preserved():
    from distributed_llm_backend_benchmark_amd.ops import cast

    x = torch.tensor([float("nan"), float("inf"), -float("inf"), 1.0, -0.0] * 4, device=DEV)
    y = cast(x, torch.bfloat16).float()
    assert torch.isnan(y[0]) and y[1] == float("inf") and y[2] == -float("inf")


@pytest.mark.parametrize("cols,ld", [(1024, 3072), (24, 72), (13, 40)])
def test_pack_rows(cols, ld):
    from distributed_llm_backend_benchmark_amd.ops import pack_rows

    base = _randn(257, ld, seed=4)
    view = base[:, :cols]
    out = pack_rows(view, dtype=torch.float32)
    torch.testing.assert_close(out, view.float(), rtol=0, atol=0)


@pytest.mark.parametrize("nt", [0, 1, 2])
def test_chunk_copy_and_scale(nt):
    from distributed_llm_backend_benchmark_amd.ops import ChunkTable, ScaleTable, _lib, flatten_into

    _lib.lib().dlbb_chunk_copy_set_nt(nt)

    ts = [_randn(n, seed=i) for i, n in enumerate([1, 7, 1024, 300001, 64])]
    flat = torch.zeros(sum(t.numel() for t in ts), dtype=torch.bfloat16, device=DEV)
    tab = flatten_into(ts, flat)
    tab.run()
    torch.testing.assert_close(flat, torch.cat(ts), rtol=0, atol=0)
    # unaligned byte copy
    a = torch.arange(1001, dtype=torch.uint8, device=DEV)
    b = torch.zeros(1001, dtype=torch.uint8, device=DEV)
    ChunkTable([(a[1:], b[:-1])]).run()
    assert torch.equal(b[:-1], a[1:])
    outs = [torch.empty(t.numel(), dtype=torch.float32, device=DEV) for t in ts]
    off, views = 0, []
    for t in ts:
        views.append(flat[off:off + t.numel()])
        off += t.numel()
    ScaleTable(list(zip(views, outs)), scale=0.125).run()
    for t, o in zip(ts, outs):
        torch.testing.assert_close(o, t.float() * 0.125, rtol=1e-6, atol=1e-6)
    if nt == 2:       # auto: a copy past the MALL size takes the non-temporal stores
        big = _randn(80 << 20, seed=9)
        dst = torch.empty_like(big)
        ChunkTable([(big, dst)]).run()
        assert torch.equal(dst, big)
    _lib.lib().dlbb_chunk_copy_set_nt(2)


@pytest.fixture(params=[("mfma", 0, 6), ("mfma", 128, 6), ("mfma", 256, 3), ("mfma", 256, 6),
                        ("mfma", 256, 6, 0), ("mfma", 256, 6, 1), ("mfma", 256, 10),
                        ("blas", 0, 6)],
                ids=["mfma_auto", "mfma_t128", "mfma_t256_deep", "mfma_t256_pingpong",
                     "mfma_t256_pingpong_nobal", "mfma_t256_pingpong_bal",
                     "mfma_t256_pp_persistent", "blas"])
def gemm_tile(request, monkeypatch):
    from distributed_llm_backend_benchmark_amd.ops.gemm import (get_stagger, set_bal, set_stagger,
                                                                set_tile)

    impl, tile, stagger = request.param[:3]
    monkeypatch.setenv("DLBB_GEMM", impl)
    old = get_stagger()
    set_tile(tile)
    set_stagger(stagger)
    set_bal(request.param[3] if len(request.param) > 3 else 2)
    yield request.param
    set_tile(0)
    set_stagger(old)
    set_bal(2)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (4096, 1024, 4096), (300, 200, 128),
                                   (8192, 768, 768), (128, 50304, 768), (520, 776, 192),
                                   (4096, 4352, 128), (2000, 9000, 64)])
def test_gemm_plain(M, N, K, gemm_tile):
    from distributed_llm_backend_benchmark_amd.ops import linear

    x = _randn(M, K, seed=1, scale=0.5)
    w = _randn(N, K, seed=2, scale=0.5)
    ref = x.float() @ w.float().t()
    y32 = linear(x, w, out_dtype=torch.float32)
    tol = 2e-3 if gemm_tile[0] == "mfma" else 2e-2     # blas path rounds to bf16 first
    torch.testing.assert_close(y32, ref, rtol=tol, atol=tol * (K ** 0.5))
    y = linear(x, w)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))


def test_gemm_asymmetric_identity(gemm_tile):
    """A = I with an asymmetric B catches a transposed C write (CDNA guide §3)."""
    from distributed_llm_backend_benchmark_amd.ops import linear

    n = 256
    eye = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    b = (torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n) % 17).to(torch.bfloat16)
    y = linear(eye, b, out_dtype=torch.float32)     # y = I @ b^T = b^T
    torch.testing.assert_close(y, b.float().t(), rtol=0, atol=0)


@pytest.mark.parametrize("act", [None, "gelu", "gelu_tanh"])
def test_gemm_epilogues(act, gemm_tile):
    from distributed_llm_backend_benchmark_amd.ops import linear

    M, N, K = 512, 384, 256
    x = _randn(M, K, seed=5, scale=0.3)
    w = _randn(N, K, seed=6, scale=0.3)
    b = _randn(N, seed=7)
    r = _randn(M, N, seed=8)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    u = x.float() @ w.float().t() + b.float()
    if act == "gelu":
        ref = F.gelu(u)
    elif act == "gelu_tanh":
        ref = F.gelu(u, approximate="tanh")
    else:
        ref = u
    ref = ref + r.float()
    y = linear(x, w, bias=b, act=act, residual=r, out_dtype=torch.float32, preact=pre)
    tol = 2e-3 if gemm_tile[0] == "mfma" else 2e-2
    torch.testing.assert_close(y, ref, rtol=tol, atol=3e-2)
    torch.testing.assert_close(pre.float(), u, rtol=1e-2, atol=3e-2)


@pytest.mark.parametrize("M,N,K,act,with_pre", [
    (16384, 2304, 768, None, False),          # GPT-2 QKV: bias, 576 tiles on 256 CUs
    (8192 + 40, 3072, 768, "gelu_tanh", True),  # GPT-2 FC (ragged last row block), preact
    (8192, 3072, 256, "gelu", True),            # erf GELU, 4 K-tiles
    (8192, 2048 + 64, 2560, "gelu_tanh", False),  # 40 K-tiles (balanced DMA), N % 256 == 64
])
@pytest.mark.parametrize("persist_epi", [True, False])
def test_gemm_persistent_lean_epilogues(M, N, K, act, with_pre, persist_epi, monkeypatch):
    """Persistent NT kernel with the bias / bias-GELU (+ pre-activation) epilogue stored at the next
    tile's first memory interval, against fp32; the non-persistent ping-pong (persist_epi off) is
    held to the same reference."""
    from distributed_llm_backend_benchmark_amd.ops import gemm, linear

    x = _randn(M, K, seed=31, scale=0.3)
    w = _randn(N, K, seed=32, scale=0.3)
    b = _randn(N, seed=33)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV) if with_pre else None
    u = x.float() @ w.float().t() + b.float()
    ref = u if act is None else F.gelu(u, approximate="tanh" if act == "gelu_tanh" else "none")
    monkeypatch.setenv("DLBB_GEMM", "mfma")
    gemm.set_persist_epi(persist_epi)
    try:
        y = linear(x, w, bias=b, act=act, preact=pre)
    finally:
        gemm.set_persist_epi(True)
    torch.cuda.synchronize()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    if with_pre:
        torch.testing.assert_close(pre.float(), u, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (16384, 768, 3072), (520, 192, 128),
                                   (4096, 2304, 64), (8, 384, 192), (1024 + 8, 1536, 4096)])
@pytest.mark.parametrize("epi", ["plain_f32", "bias_res", "bias_gelu_pre", "plain_bf16"])
@pytest.mark.parametrize("bal", [0, 1])
def test_gemm_nt_192_tiles_match_fp32(M, N, K, epi, bal, monkeypatch):
    """256 x 192 ping-pong tiles (variant 1, the partial-round fix for N % 192 == 0) against an
    fp32 reference: ragged M, 1 .. 64 K-tiles, every epilogue (bias, residual, GELU with the
    pre-activation store, fp32 / bf16 output), plain and balanced DMA issue."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    x = _randn(M, K, seed=41, scale=0.3)
    w = _randn(N, K, seed=42, scale=0.3)
    b = _randn(N, seed=43)
    r = _randn(M, N, seed=44)
    u = x.float() @ w.float().t()
    gemm.set_bal(bal)
    try:
        if epi == "plain_f32":
            y = torch.empty(M, N, dtype=torch.float32, device=DEV)
            gemm._mfma192_linear(x, w, None, None, None, y, None)
            torch.testing.assert_close(y, u, rtol=2e-3, atol=2e-3 * K ** 0.5)
        elif epi == "plain_bf16":
            y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm._mfma192_linear(x, w, None, None, None, y, None)
            torch.testing.assert_close(y.float(), u, rtol=2e-2, atol=2e-2 * K ** 0.5)
        elif epi == "bias_res":
            y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm._mfma192_linear(x, w, b, None, r, y, None)
            torch.testing.assert_close(y.float(), u + b.float() + r.float(), rtol=2e-2,
                                       atol=2e-2 * K ** 0.5)
        else:
            y = torch.empty(M, N, dtype=torch.float32, device=DEV)
            pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm._mfma192_linear(x, w, b, "gelu_tanh", None, y, pre)
            ub = u + b.float()
            torch.testing.assert_close(y, F.gelu(ub, approximate="tanh"), rtol=2e-3,
                                       atol=2e-3 * K ** 0.5)
            torch.testing.assert_close(pre.float(), ub, rtol=2e-2, atol=2e-2 * K ** 0.5)
    finally:
        gemm.set_bal(2)
    torch.cuda.synchronize()


def test_gemm_strided_A_view():
    """The TP attention stub passes qkv[..., :H/P] (lda = 3H/P) straight into the GEMM."""
    from distributed_llm_backend_benchmark_amd.ops import linear

    qkv = _randn(256, 3 * 512, seed=9, scale=0.3)
    a = qkv[:, :512]
    w = _randn(640, 512, seed=10, scale=0.3)
    torch.testing.assert_close(linear(a, w, out_dtype=torch.float32),
                               a.float() @ w.float().t(), rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (16384, 768, 2304), (520, 512, 192),
                                   (8, 256, 64), (1000, 3072, 768), (2048, 768, 50304),
                                   (4096, 4096, 4096)])
@pytest.mark.parametrize("bal", [0, 1])
def test_dgrad_nn_matches_fp32(M, N, K, bal):
    """NN kernel (transposed-read W): dX = dY @ W against an fp32 reference; ragged M, one
    K-tile, LM-head-sized reduction; plain and balanced DMA issue."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    dy = _randn(M, K, seed=21, scale=0.5)
    w = _randn(K, N, seed=22, scale=0.5)
    assert gemm.dgrad_supported(dy, w)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    gemm.set_bal(bal)
    try:
        gemm._dgrad_hip(dy, w, out)
    finally:
        gemm.set_bal(2)
    ref = dy.float() @ w.float()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))


@pytest.mark.parametrize("T,N,K,bal", [(1024, 384, 768, 2), (64, 256, 256, 0), (2048, 640, 512, 1),
                                       (16384, 896, 768, 2)])
def test_wgrad_pingpong_tn_matches_fp32(T, N, K, bal):
    """256^2 ping-pong weight gradient (both operands transposed-read images): dW = dY^T X
    against an fp32 reference; output rows ragged by half a tile (N % 256 == 128: the second A
    image re-staged, never stored), one K-tile, the GPT-2 token count; plain and balanced."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    dy = _randn(T, N, seed=41, scale=0.5)
    x = _randn(T, K, seed=42, scale=0.5)
    out = torch.full((N, K), float("nan"), dtype=torch.bfloat16, device=DEV)
    assert gemm.wgrad_pp_supported(dy, x, out, False)
    gemm.set_bal(bal)
    try:
        gemm._wgrad_pp(dy, x, out, False)
    finally:
        gemm.set_bal(2)
    ref = dy.float().t() @ x.float()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2 * (T ** 0.5))
    # accumulate (bf16 out, residual = out) and fp32 output
    acc = out.clone()
    gemm._wgrad_pp(dy, x, acc, True)
    torch.testing.assert_close(acc.float(), 2 * ref, rtol=3e-2, atol=4e-2 * (T ** 0.5))
    o32 = torch.empty(N, K, dtype=torch.float32, device=DEV)
    gemm._wgrad_pp(dy, x, o32, False)
    torch.testing.assert_close(o32, ref, rtol=1e-3, atol=1e-3 * (T ** 0.5))


@pytest.mark.parametrize("T,N,K,r0,split", [(1024, 384, 512, 0, 3), (2048, 896, 768, 256, 4),
                                             (4096, 640, 256, 128, 2),
                                             # 10 K-tiles, split 7 -> 2 per slice: the launch
                                             # clamps to 5 slices (7 would start 2 past K)
                                             (640, 256, 256, 0, 7)])
def test_wgrad_pingpong_tn_split_k(T, N, K, r0, split):
    """TN split-K on a row range [r0, N) (the LM-head tail path): uneven K slices (16 / 3 K-tiles),
    a row offset into dY, fp32 partials + reduce; rows outside the range untouched."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    dy = _randn(T, N, seed=43, scale=0.5)
    x = _randn(T, K, seed=44, scale=0.5)
    out = torch.full((N, K), 7.0, dtype=torch.bfloat16, device=DEV)
    gemm._pp_launch(dy, x, out, False, r0, N, split)
    ref = dy.float().t() @ x.float()
    torch.testing.assert_close(out[r0:].float(), ref[r0:], rtol=2e-2, atol=2e-2 * (T ** 0.5))
    assert bool((out[:r0] == 7.0).all())


@pytest.mark.parametrize("T,N,K,split", [(16384, 3072, 768, None), (16384, 768, 3072, None),
                                         (16384, 768, 768, None), (2048, 256, 512, 3),
                                         (1024, 128, 256, 1)])
def test_wgrad_wide_matches_fp32(T, N, K, split):
    """128 x 256 weight-gradient tiles (4 waves of 64 x 128): dW and the fused bias gradient
    against fp32; split-K reduce, one split with a direct store, accumulate into bf16 and fp32."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    dy = _randn(T, N, seed=51, scale=0.5)
    x = _randn(T, K, seed=52, scale=0.5)
    ref = dy.float().t() @ x.float()
    rb = dy.float().sum(0)
    out = torch.full((N, K), float("nan"), dtype=torch.bfloat16, device=DEV)
    db = torch.full((N,), float("nan"), dtype=torch.bfloat16, device=DEV)
    gemm._wgrad_hip_wide(dy, x, out, False, split, db)
    tol = 2e-2 * (T ** 0.5)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=tol)
    torch.testing.assert_close(db.float(), rb, rtol=2e-2, atol=tol)
    plain = torch.full((N, K), float("nan"), dtype=torch.bfloat16, device=DEV)
    gemm._wgrad_hip_wide(dy, x, plain, False, split)          # no bias (direct store at split 1)
    torch.testing.assert_close(plain.float(), ref, rtol=2e-2, atol=tol)
    o32 = torch.ones(N, K, dtype=torch.float32, device=DEV)
    gemm._wgrad_hip_wide(dy, x, o32, True, split)
    torch.testing.assert_close(o32, ref + 1, rtol=1e-2, atol=1e-2 * (T ** 0.5))


def test_wgrad_pingpong_tn_tail_plan_lmhead_scale():
    """Whole rounds + split-K tail (grid 300 tiles on the device's CUs): matches fp32, and the
    plan splits it."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    ncu = torch.cuda.get_device_properties(DEV).multi_processor_count
    T, K = 1024, 256
    N = (ncu + 44) * 256                 # one whole round + a 44-tile tail
    head, split = gemm.pp_tail_plan(T, N, K, ncu)
    assert head < N and split >= 2
    dy = _randn(T, N, seed=45, scale=0.5)
    x = _randn(T, K, seed=46, scale=0.5)
    out = torch.empty(N, K, dtype=torch.bfloat16, device=DEV)
    gemm._wgrad_pp(dy, x, out, False)
    ref = dy.float().t() @ x.float()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2 * (T ** 0.5))


@pytest.mark.parametrize("M,N,K,split", [(2048, 768, 50304, 4), (520, 512, 64 * 7, 3),
                                         (1024, 256, 4096, 2),
                                         (512, 256, 64 * 10, 7)])   # clamped to 5 slices
def test_dgrad_nn_split_k(M, N, K, split):
    """Split-K NN (uneven last slice for 786 / 4 and 7 / 3 K-tiles): fp32 partials + reduce."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    dy = _randn(M, K, seed=27, scale=0.5)
    w = _randn(K, N, seed=28, scale=0.5)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    gemm._dgrad_hip(dy, w, out, split=split)
    ref = dy.float() @ w.float()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))
    assert gemm.dgrad_split(16384, 768, 50304) == 4 and gemm.dgrad_split(16384, 768, 3072) == 1


def test_dgrad_nn_asymmetric_identity_and_strided():
    """A = I with an asymmetric W catches any column permutation (the JSWAP epilogue) or a
    transposed write; a strided dY view (lda > K) checks the A panel addressing."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    n = 512
    eye = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    w = (torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n) % 61).to(torch.bfloat16)
    out = torch.empty(n, n, dtype=torch.bfloat16, device=DEV)
    gemm._dgrad_hip(eye, w, out)
    torch.testing.assert_close(out.float(), w.float(), rtol=0, atol=0)
    big = _randn(768, 3 * 256, seed=23, scale=0.5)
    dy = big[:, :256]
    w2 = _randn(256, 1024, seed=24, scale=0.5)
    out2 = torch.empty(768, 1024, dtype=torch.bfloat16, device=DEV)
    gemm._dgrad_hip(dy, w2, out2)
    torch.testing.assert_close(out2.float(), dy.float() @ w2.float(), rtol=2e-2, atol=2e-2 * 16)


def test_dgrad_dispatch_counts_hand_written():
    from distributed_llm_backend_benchmark_amd.ops import gemm

    dy = _randn(4096, 1024, seed=25, scale=0.5)
    w = _randn(1024, 768, seed=26, scale=0.5)
    y = gemm.dgrad(dy, w)
    torch.testing.assert_close(y.float(), dy.float() @ w.float(), rtol=2e-2, atol=2e-2 * 32)
    assert (4096, 768, 1024, 1024, None) in gemm.DGRAD_CHOICES
    mix = gemm.kernel_mix()
    assert "dgrad" in mix and mix["dgrad"]["tuned"]


@pytest.mark.parametrize("cols", [256, 768, 2048, 4096, 5120, 8192, 100])
@pytest.mark.parametrize("with_res", [False, True])
def test_layernorm_fwd(cols, with_res):
    from distributed_llm_backend_benchmark_amd.ops import layernorm

    rows = 333
    x = _randn(rows, cols, seed=11, scale=2.0)
    r = _randn(rows, cols, seed=12) if with_res else None
    w = _randn(cols, seed=13)
    b = _randn(cols, seed=14)
    y, h = layernorm(x, w, b, 1e-5, residual=r)
    hin = (x.float() + r.float()).to(torch.bfloat16).float() if with_res else x.float()
    ref = F.layer_norm(hin, (cols,), w.float(), b.float(), 1e-5)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=3e-2)
    if with_res:
        torch.testing.assert_close(h.float(), hin, rtol=0, atol=0)


@pytest.mark.parametrize("cols", [768, 1024, 4096, 128, 200])
@pytest.mark.parametrize("with_res", [False, True])
def test_layernorm_bwd(cols, with_res):
    """Fused backward at the instantiated widths; at others (128, 200: toy models) the same math
    in fp32 torch ops, counted in ``LN_FALLBACKS``."""
    from distributed_llm_backend_benchmark_amd.ops import layernorm
    from distributed_llm_backend_benchmark_amd.ops import norm_act

    fb0 = norm_act.LN_FALLBACKS["count"]

    rows = 520
    x = _randn(rows, cols, seed=15).requires_grad_(True)
    r = _randn(rows, cols, seed=16).requires_grad_(True) if with_res else None
    w = _randn(cols, seed=17).requires_grad_(True)
    b = _randn(cols, seed=18).requires_grad_(True)
    dy = _randn(rows, cols, seed=19)
    dh = _randn(rows, cols, seed=20) if with_res else None
    y, h = layernorm(x, w, b, 1e-5, residual=r)
    loss = (y.float() * dy.float()).sum()
    if with_res:
        loss = loss + (h.float() * dh.float()).sum()
    loss.backward()
    # fp32 reference
    xf = x.detach().float().requires_grad_(True)
    rf = r.detach().float().requires_grad_(True) if with_res else None
    wf = w.detach().float().requires_grad_(True)
    bf = b.detach().float().requires_grad_(True)
    hf = xf + rf if with_res else xf
    yf = F.layer_norm(hf, (cols,), wf, bf, 1e-5)
    lf = (yf * dy.float()).sum() + ((hf * dh.float()).sum() if with_res else 0)
    lf.backward()
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(w.grad.float(), wf.grad, rtol=3e-2, atol=0.5)
    torch.testing.assert_close(b.grad.float(), bf.grad, rtol=3e-2, atol=0.5)
    if with_res:
        torch.testing.assert_close(r.grad.float(), rf.grad, rtol=3e-2, atol=3e-2)
    assert norm_act.LN_FALLBACKS["count"] - fb0 == (0 if cols % 256 == 0 else 1)


@pytest.mark.parametrize("rows,cols", [(16384, 768), (520, 768), (4099, 1024), (7, 256),
                                       (1000, 2048)])
@pytest.mark.parametrize("with_res", [False, True])
def test_layernorm_bwd_matches_fp32(rows, cols, with_res):
    """The LN backward (pipelined kernel up to 1024 columns, the wave-per-row-sequence kernel
    beyond) against the fp32 torch reference: dx, dgamma, dbeta (+ the residual gradient)."""
    from distributed_llm_backend_benchmark_amd.ops import _lib
    from distributed_llm_backend_benchmark_amd.ops.norm_act import _ln_bwd_reference

    L = _lib.lib()
    h, dy = _randn(rows, cols, seed=31), _randn(rows, cols, seed=32)
    dres = _randn(rows, cols, seed=33) if with_res else None
    gam = _randn(cols, seed=34)
    mean = h.float().mean(1)
    rstd = torch.rsqrt(h.float().var(1, unbiased=False) + 1e-5)
    grid = L.dlbb_layernorm_bwd_grid(rows)
    dx = torch.empty_like(h)
    ws = torch.full((2 * grid * cols,), float("nan"), device=DEV)
    dg = torch.empty(cols, device=DEV, dtype=torch.bfloat16)
    db = torch.empty(cols, device=DEV, dtype=torch.bfloat16)
    _lib.check(L.dlbb_layernorm_bwd(
        dy.data_ptr(), h.data_ptr(), gam.data_ptr(), 1, mean.data_ptr(), rstd.data_ptr(),
        _lib.ptr(dres), dx.data_ptr(), ws.data_ptr(), dg.data_ptr(), db.data_ptr(), rows,
        cols, 0, _lib.stream(h.device)), "ln_bwd")
    rdg, rdb = torch.empty(cols, device=DEV), torch.empty(cols, device=DEV)
    rdx = _ln_bwd_reference(dy, h, gam, mean, rstd, dres, rdg, rdb, False)
    torch.testing.assert_close(dx.float(), rdx.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dg.float(), rdg, rtol=1e-2, atol=1e-2 * rows ** 0.5)
    torch.testing.assert_close(db.float(), rdb, rtol=1e-2, atol=1e-2 * rows ** 0.5)


@pytest.mark.parametrize("approx", ["none", "tanh"])
def test_bias_gelu_fwd_bwd(approx):
    from distributed_llm_backend_benchmark_amd.ops import bias_gelu

    rows, cols = 700, 3072
    x = _randn(rows, cols, seed=21, scale=2.0).requires_grad_(True)
    b = _randn(cols, seed=22).requires_grad_(True)
    dy = _randn(rows, cols, seed=23)
    y = bias_gelu(x, b, approximate=approx)
    (y.float() * dy.float()).sum().backward()
    xf = x.detach().float().requires_grad_(True)
    bf = b.detach().float().requires_grad_(True)
    yf = F.gelu(xf + bf, approximate=approx)
    (yf * dy.float()).sum().backward()
    torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(b.grad.float(), bf.grad, rtol=2e-2, atol=0.5)


@pytest.mark.parametrize("act", ["gelu_tanh", None])
def test_linear_train_grads(act):
    from distributed_llm_backend_benchmark_amd.ops.linear_fn import linear_train

    M, N, K = 512, 1024, 256
    x = _randn(M, K, seed=24, scale=0.5).requires_grad_(True)
    w = _randn(N, K, seed=25, scale=0.1).requires_grad_(True)
    b = _randn(N, seed=26).requires_grad_(True)
    dy = _randn(M, N, seed=27)
    y = linear_train(x, w, b, act=act)
    (y.float() * dy.float()).sum().backward()
    xf, wf, bf = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yf = xf @ wf.t() + bf
    if act:
        yf = F.gelu(yf, approximate="tanh")
    (yf * dy.float()).sum().backward()
    torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=3e-2, atol=0.2)
    torch.testing.assert_close(w.grad.float(), wf.grad, rtol=3e-2, atol=0.5)
    torch.testing.assert_close(b.grad.float(), bf.grad, rtol=3e-2, atol=0.5)


@pytest.mark.parametrize("act", ["gelu_tanh", "gelu"])
@pytest.mark.parametrize("impl", ["mfma", "blas"])
def test_dgrad_fused_gelu_backward(act, impl, monkeypatch):
    """dgrad epilogue (dY @ W) * act'(u) vs fp32, through both dispatch paths."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    monkeypatch.setenv("DLBB_GEMM", impl)
    M, N, K = 1024, 3072, 768
    dy = _randn(M, K, seed=31, scale=0.5)
    w = _randn(K, N, seed=32, scale=0.05)
    u = _randn(M, N, seed=33, scale=2.0)
    out = gemm.dgrad(dy, w, dgelu=(u, act))
    uf = u.float().requires_grad_(True)
    g = F.gelu(uf, approximate="tanh" if act == "gelu_tanh" else "none")
    g.backward(dy.float() @ w.float())
    torch.testing.assert_close(out.float(), uf.grad, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("M,N,K,act", [(16384, 3072, 768, "gelu_tanh"), (8192 + 40, 2048, 512, "gelu"),
                                       (16384, 3072, 768, None), (4096 + 8, 4096, 2048, None)])
@pytest.mark.parametrize("persist", [True, False])
def test_dgrad_persistent_matches_fp32(M, N, K, act, persist):
    """NN dgrad on multi-round short-K grids: the persistent form (plain / GELU backward with the
    epilogue's u read at the tile boundary; ragged last row block) and the non-persistent ping-pong
    against fp32."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    dy = _randn(M, K, seed=41, scale=0.5)
    w = _randn(K, N, seed=42, scale=0.05)
    u = _randn(M, N, seed=43, scale=2.0) if act else None
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    gemm.set_persist_epi(persist)
    try:
        gemm._dgrad_hip(dy, w, out, None, (u, act) if act else None)
    finally:
        gemm.set_persist_epi(True)
    g = dy.float() @ w.float()
    if act:
        uf = u.float().requires_grad_(True)
        F.gelu(uf, approximate="tanh" if act == "gelu_tanh" else "none").backward(g)
        g = uf.grad
    torch.testing.assert_close(out.float(), g, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("sinks", [False, True])
def test_mlp_train_grads(sinks):
    """Fused MLP op (GELU backward in the dgrad epilogue) vs an fp32 autograd reference; with
    gradient sinks the weight gradients land in the parameters' .grad buffers in-kernel."""
    from distributed_llm_backend_benchmark_amd.ops.linear_fn import mlp_train

    M, C, H = 512, 256, 1024
    x = _randn(M, C, seed=34, scale=0.5).requires_grad_(True)
    w1 = _randn(H, C, seed=35, scale=0.05).requires_grad_(True)
    b1 = _randn(H, seed=36, scale=0.1).requires_grad_(True)
    w2 = _randn(C, H, seed=37, scale=0.05).requires_grad_(True)
    b2 = _randn(C, seed=38, scale=0.1).requires_grad_(True)
    params = (w1, b1, w2, b2)
    fired = []
    if sinks:
        for p in params:
            p.grad = torch.zeros_like(p)
            p._dlbb_grad_fresh = True
            p._dlbb_grad_sink = fired.append
    dy = _randn(M, C, seed=39)
    y = mlp_train(x, w1, b1, w2, b2, act="gelu_tanh")
    (y.float() * dy.float()).sum().backward()
    xf, w1f, b1f, w2f, b2f = (t.detach().float().requires_grad_(True) for t in (x, *params))
    yf = F.gelu(xf @ w1f.t() + b1f, approximate="tanh") @ w2f.t() + b2f
    (yf * dy.float()).sum().backward()
    torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=3e-2, atol=0.1)
    for p, pf in zip(params, (w1f, b1f, w2f, b2f)):
        torch.testing.assert_close(p.grad.float(), pf.grad, rtol=3e-2, atol=0.3)
    if sinks:
        assert len(fired) == 4


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_adamw(gdt):
    from distributed_llm_backend_benchmark_amd.ops import FlatAdamW

    n = 100003
    p = _randn(n, dtype=torch.float32, seed=28)
    pref = p.clone().requires_grad_(True)
    opt = FlatAdamW(p, lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    ref = torch.optim.AdamW([pref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    shadow = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    for s in range(3):
        g = _randn(n, dtype=gdt, seed=100 + s)
        opt.step(g, working_bf16=shadow, grad_scale=0.5)
        pref.grad = g.float() * 0.5
        ref.step()
    torch.testing.assert_close(p, pref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(shadow, p.to(torch.bfloat16), rtol=0, atol=0)


@pytest.mark.parametrize("V", [50304, 1000])
def test_cross_entropy_fwd_bwd(V):
    from distributed_llm_backend_benchmark_amd.ops import cross_entropy

    rows = 300
    x = _randn(rows, V, seed=40, scale=3.0).requires_grad_(True)
    t = torch.randint(0, V, (rows,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    t[::7] = -100                       # ignore_index rows
    loss = cross_entropy(x, t)
    loss.backward()
    xf = x.detach().float().requires_grad_(True)
    lf = F.cross_entropy(xf, t, ignore_index=-100)
    lf.backward()
    torch.testing.assert_close(loss.float(), lf, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=2e-2, atol=2e-5)


@pytest.mark.parametrize("V,gscale", [(50304, 1.0), (1000, 3.0), (2048, 1.0)])
def test_linear_cross_entropy_fused(V, gscale):
    """LM head + loss fused (one in-place pass turns logits into loss and dlogits) against the
    fp32 torch reference of linear + cross-entropy: loss, dX and dW, with ignore_index rows and
    an upstream gradient != 1."""
    from distributed_llm_backend_benchmark_amd.ops import linear_cross_entropy

    rows, K = 512, 256
    x = _randn(rows, K, seed=41, scale=1.0).requires_grad_(True)
    w = _randn(V, K, seed=42, scale=0.05).requires_grad_(True)
    t = torch.randint(0, V, (rows,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
    t[::5] = -100
    loss = linear_cross_entropy(x, w, t)
    (loss * gscale).backward()
    xf = x.detach().float().requires_grad_(True)
    wf = w.detach().float().requires_grad_(True)
    lf = F.cross_entropy(xf @ wf.t(), t, ignore_index=-100)
    (lf * gscale).backward()
    torch.testing.assert_close(loss.float(), lf, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=3e-2, atol=3e-4 * gscale)
    torch.testing.assert_close(w.grad.float(), wf.grad, rtol=3e-2, atol=3e-4 * gscale)


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("V", [50304, 1000, 4096 * 8 + 8])
def test_xent_fused_pass_elementwise(V, variant):
    """The in-place fused loss pass itself: every dlogit against fp32 (softmax - onehot) * scale
    and every row loss, with targets on the first / last column / a vector boundary and
    ignore_index rows; both kernel variants (v2 default, v1 kept for A/B)."""
    from distributed_llm_backend_benchmark_amd.ops import _lib as L

    rows = 96
    x = _randn(rows, V, seed=43, scale=4.0)
    t = torch.randint(0, V, (rows,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    t[0], t[1], t[2], t[3] = 0, V - 1, 7, 8
    t[5::9] = -100
    sc = torch.full((1,), 0.37, device=DEV)
    loss = torch.empty(rows, device=DEV)
    buf = x.clone()
    L.lib().dlbb_xent_set_variant(variant)
    try:
        L.check(L.lib().dlbb_xent_fused(buf.data_ptr(), t.data_ptr(), loss.data_ptr(), rows, V, V,
                                        sc.data_ptr(), L.stream(buf.device)), "xent_fused")
        torch.cuda.synchronize()
    finally:
        L.lib().dlbb_xent_set_variant(2)
    xf = x.float()
    valid = t >= 0
    lse = torch.logsumexp(xf, dim=1)
    ref_loss = torch.where(valid, lse - xf.gather(1, t.clamp_min(0)[:, None])[:, 0],
                           torch.zeros_like(lse))
    p = torch.softmax(xf, dim=1)
    p[valid, t[valid]] -= 1.0
    ref = p * 0.37 * valid[:, None].float()
    torch.testing.assert_close(loss, ref_loss, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(buf.float(), ref, rtol=1.6e-2, atol=1e-6)


@pytest.mark.parametrize("M,N,K", [(64, 128, 128), (16384, 768, 768), (4096, 2304, 768),
                                   (1024, 256, 3072), (320, 384, 256), (96, 128, 256)])
@pytest.mark.parametrize("split", [None, 1, 3])
def test_wgrad_matches_fp32(M, N, K, split):
    from distributed_llm_backend_benchmark_amd.ops.gemm import wgrad

    dy = _randn(M, N, seed=21, scale=0.5)
    x = _randn(M, K, seed=22, scale=0.5)
    ref = dy.float().t() @ x.float()
    out32 = torch.empty(N, K, dtype=torch.float32, device=DEV)
    wgrad(dy, x, out=out32, split=split)
    torch.testing.assert_close(out32, ref, rtol=2e-3, atol=2e-3 * (M ** 0.5))
    acc = torch.ones(N, K, dtype=torch.float32, device=DEV)
    wgrad(dy, x, out=acc, accumulate=True, split=split)
    torch.testing.assert_close(acc, ref + 1, rtol=2e-3, atol=2e-3 * (M ** 0.5))
    y = wgrad(dy, x, split=split)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * (M ** 0.5))
    # fused bias gradient (all-ones MFMA operand in the column-block-0 workgroups)
    refb = dy.float().sum(0)
    w32, b32 = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
    wgrad(dy, x, out=w32, split=split, bias_out=b32)
    torch.testing.assert_close(w32, ref, rtol=2e-3, atol=2e-3 * (M ** 0.5))
    torch.testing.assert_close(b32, refb, rtol=2e-3, atol=2e-3 * (M ** 0.5))
    b32.fill_(1.0)
    wgrad(dy, x, out=w32, accumulate=True, split=split, bias_out=b32)
    torch.testing.assert_close(b32, refb + 1, rtol=2e-3, atol=2e-3 * (M ** 0.5))


@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (4096, 2304, 768), (1024, 256, 3072)])
def test_wgrad_forced_pp_with_bias(monkeypatch, M, N, K):
    """DLBB_GEMM=pp: the unsplit 256^2 TN ping-pong for dW plus a column-sum pass for the
    bias gradient (the kernel has no fused bias): bf16 store and bf16 accumulate."""
    from distributed_llm_backend_benchmark_amd.ops import gemm as G

    monkeypatch.setenv("DLBB_GEMM", "pp")
    dy = _randn(M, N, seed=31, scale=0.5)
    x = _randn(M, K, seed=32, scale=0.5)
    assert G._wgrad_choice(dy, x, torch.empty(N, K, dtype=torch.bfloat16, device=DEV),
                           torch.empty(N, dtype=torch.bfloat16, device=DEV)) == "pp"
    ref = dy.float().t() @ x.float()
    refb = dy.float().sum(0)
    w = torch.empty(N, K, dtype=torch.bfloat16, device=DEV)
    b = torch.empty(N, dtype=torch.bfloat16, device=DEV)
    G.wgrad(dy, x, out=w, bias_out=b)
    torch.testing.assert_close(w.float(), ref, rtol=2e-2, atol=2e-2 * (M ** 0.5))
    torch.testing.assert_close(b.float(), refb, rtol=2e-2, atol=2e-2 * (M ** 0.5))
    w.fill_(1.0)
    b.fill_(1.0)
    G.wgrad(dy, x, out=w, accumulate=True, bias_out=b)
    torch.testing.assert_close(w.float(), ref + 1, rtol=2e-2, atol=2e-2 * (M ** 0.5))
    torch.testing.assert_close(b.float(), refb + 1, rtol=2e-2, atol=2e-2 * (M ** 0.5))


@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (4096, 2304, 768), (1024, 256, 3072),
                                   (512, 3072, 768), (96, 512, 128)])
@pytest.mark.parametrize("split", [None, 1, 3])
def test_wgrad_256_tile_matches_fp32(M, N, K, split):
    """The 256 x 128 output tile (8 waves, two A sub-images per stage): dW, accumulate and the
    fused bias gradient against fp32."""
    from distributed_llm_backend_benchmark_amd.ops.gemm import _wgrad_hip256

    dy = _randn(M, N, seed=51, scale=0.5)
    x = _randn(M, K, seed=52, scale=0.5)
    ref = dy.float().t() @ x.float()
    refb = dy.float().sum(0)
    tol = dict(rtol=2e-3, atol=2e-3 * (M ** 0.5))
    w32, b32 = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
    _wgrad_hip256(dy, x, w32, False, split, None)
    torch.testing.assert_close(w32, ref, **tol)
    _wgrad_hip256(dy, x, w32, False, split, b32)
    torch.testing.assert_close(w32, ref, **tol)
    torch.testing.assert_close(b32, refb, **tol)
    w32.fill_(1.0)
    b32.fill_(1.0)
    _wgrad_hip256(dy, x, w32, True, split, b32)
    torch.testing.assert_close(w32, ref + 1, **tol)
    torch.testing.assert_close(b32, refb + 1, **tol)
    wb = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
    _wgrad_hip256(dy, x, wb, False, split, None)
    torch.testing.assert_close(wb.float(), ref, rtol=2e-2, atol=2e-2 * (M ** 0.5))


@pytest.mark.parametrize("impl", ["mfma", "mfma256", "mfma_wide"])
@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (16384, 3072, 768), (4096, 2304, 768),
                                   (512, 768, 3072)])
@pytest.mark.parametrize("order", [0, 1])
def test_wgrad_fused_reduce_bitwise(monkeypatch, impl, M, N, K, order):
    """In-launch split-K combine (last-arriving workgroup per tile) against the separate reduce
    pass: same fp32 summation order, so dW / db / accumulate results must be BITWISE equal, for
    both workgroup orders (a tile's slices on one XCD, or spread over all of them)."""
    from distributed_llm_backend_benchmark_amd.ops import _lib, gemm

    fn = {"mfma": gemm._wgrad_hip, "mfma256": gemm._wgrad_hip256,
          "mfma_wide": gemm._wgrad_hip_wide}[impl]
    if impl == "mfma256" and N % 256 or impl == "mfma_wide" and K % 256:
        pytest.skip("tile does not divide the shape")
    dy = _randn(M, N, seed=61, scale=0.5)
    x = _randn(M, K, seed=62, scale=0.5)
    _lib.lib().dlbb_gemm_wgrad_set_order(order)
    try:
        outs = {}
        for fused in ("0", "1"):
            monkeypatch.setattr(gemm, "_WGRAD_FUSED", [fused == "1"])
            w32, b32 = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
            fn(dy, x, w32, False, None, b32)
            wacc, bacc = torch.full((N, K), 0.25, device=DEV), torch.full((N,), 0.5, device=DEV)
            fn(dy, x, wacc, True, None, bacc)
            wb = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
            bb = torch.empty(N, device=DEV, dtype=torch.bfloat16)
            fn(dy, x, wb, False, None, bb)
            outs[fused] = (w32, b32, wacc, bacc, wb, bb)
        for a, b in zip(outs["0"], outs["1"]):
            assert torch.equal(a, b)
        ref = dy.float().t() @ x.float()
        torch.testing.assert_close(outs["1"][0], ref, rtol=2e-3, atol=2e-3 * (M ** 0.5))
        torch.testing.assert_close(outs["1"][1], dy.float().sum(0), rtol=2e-3,
                                   atol=2e-3 * (M ** 0.5))
    finally:
        _lib.lib().dlbb_gemm_wgrad_set_order(1)


def test_wgrad_fused_reduce_repeated_under_load(monkeypatch):
    """20 back-to-back fused launches on one stream with different inputs while a second stream
    streams HBM (uneven load, reducer L1 warm from the previous launch): every result must equal
    the separate-pass result, and the per-stream tile counters end at zero (re-armed)."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    M, N, K = 16384, 768, 768
    xs = [_randn(M, K, seed=70 + i, scale=0.5) for i in range(4)]
    dys = [_randn(M, N, seed=80 + i, scale=0.5) for i in range(4)]
    monkeypatch.setattr(gemm, "_WGRAD_FUSED", [False])
    refs = []
    for i in range(4):
        o = torch.empty(N, K, device=DEV)
        gemm._wgrad_hip(dys[i], xs[i], o, False, None, None)
        refs.append(o)
    monkeypatch.setattr(gemm, "_WGRAD_FUSED", [True])
    side = torch.cuda.Stream()
    big = torch.empty(256 << 20, dtype=torch.uint8, device=DEV)
    outs = [torch.empty(N, K, device=DEV) for _ in range(20)]
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        for _ in range(8):
            big.add_(1)
    for i in range(20):
        gemm._wgrad_hip(dys[i % 4], xs[i % 4], outs[i], False, None, None)
    torch.cuda.synchronize()
    for i in range(20):
        assert torch.equal(outs[i], refs[i % 4]), i
    cnt = gemm._tile_counters(torch.device(DEV), 1)
    assert int(cnt.abs().sum()) == 0


def test_wgrad_256_tile_asymmetric():
    """One-hot dY columns through the 256-row tile: every dW row must be the right X row."""
    from distributed_llm_backend_benchmark_amd.ops.gemm import _wgrad_hip256

    M, N, K = 256, 512, 256
    dy = torch.zeros(M, N, device=DEV)
    dy[torch.arange(M), (torch.arange(M) * 7) % N] = 1.0
    x = (torch.arange(M * K, device=DEV, dtype=torch.float32).view(M, K) % 13)
    dy, x = dy.to(torch.bfloat16), x.to(torch.bfloat16)
    out = torch.empty(N, K, dtype=torch.float32, device=DEV)
    _wgrad_hip256(dy, x, out, False, None, None)
    torch.testing.assert_close(out, dy.float().t() @ x.float(), rtol=0, atol=0)


def test_wgrad_asymmetric():
    """dY = one-hot columns: dW rows must be the right X rows (catches swapped maps)."""
    from distributed_llm_backend_benchmark_amd.ops.gemm import wgrad

    M, N, K = 128, 128, 128
    dy = torch.zeros(M, N, device=DEV)
    dy[torch.arange(M), (torch.arange(M) * 7) % N] = 1.0
    x = (torch.arange(M * K, device=DEV, dtype=torch.float32).view(M, K) % 13)
    dy, x = dy.to(torch.bfloat16), x.to(torch.bfloat16)
    out = torch.empty(N, K, dtype=torch.float32, device=DEV)
    wgrad(dy, x, out=out)
    torch.testing.assert_close(out, dy.float().t() @ x.float(), rtol=0, atol=0)


def test_linear_train_frozen_weight_bias_grad():
    """Weight frozen, bias trained: db cannot ride on the (skipped) wgrad kernels."""
    from distributed_llm_backend_benchmark_amd.ops.linear_fn import linear_train

    M, N, K = 256, 512, 256
    x = _randn(M, K, seed=34, scale=0.5).requires_grad_(True)
    w = _randn(N, K, seed=35, scale=0.1)
    for act in (None, "gelu_tanh"):
        b = _randn(N, seed=36).requires_grad_(True)
        dy = _randn(M, N, seed=37)
        y = linear_train(x, w, b, act=act)
        (y.float() * dy.float()).sum().backward()
        bf = b.detach().float().requires_grad_(True)
        yf = x.detach().float() @ w.float().t() + bf
        if act:
            yf = F.gelu(yf, approximate="tanh")
        (yf * dy.float()).sum().backward()
        torch.testing.assert_close(b.grad.float(), bf.grad, rtol=3e-2, atol=0.5)


@pytest.mark.parametrize("B,T,Tmax,V,C", [(4, 64, 64, 50, 768), (2, 100, 128, 1000, 256)])
def test_embedding_fwd_bwd(B, T, Tmax, V, C):
    """Fused token + position embedding: forward and both gradients against fp32 torch, with
    many repeated ids (V small) and T < block size (rows >= T of the position grad stay 0)."""
    from distributed_llm_backend_benchmark_amd.ops import embedding

    g = torch.Generator(device=DEV).manual_seed(5)
    idx = torch.randint(0, V, (B, T), device=DEV, generator=g)
    wte = _randn(V, C, seed=70).requires_grad_(True)
    wpe = _randn(Tmax, C, seed=71).requires_grad_(True)
    dy = _randn(B, T, C, seed=72)
    y = embedding(idx, wte, wpe)
    y.backward(dy)
    wtef = wte.detach().float().requires_grad_(True)
    wpef = wpe.detach().float().requires_grad_(True)
    yf = F.embedding(idx, wtef) + wpef[:T]
    yf.backward(dy.float())
    torch.testing.assert_close(y.float(), yf, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(wte.grad.float(), wtef.grad, rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(wpe.grad.float(), wpef.grad, rtol=1e-2, atol=2e-2)


def test_embedding_backward_into_sinks_deterministic():
    """Sink path: gradients accumulate into preset .grad buffers (bf16), the callback fires once
    after the declared number of uses, and two runs are bitwise identical (sorted runs, no
    atomics)."""
    from distributed_llm_backend_benchmark_amd.ops import embedding

    B, T, V, C = 8, 128, 300, 512
    g = torch.Generator(device=DEV).manual_seed(6)
    idx = torch.randint(0, V, (B, T), device=DEV, generator=g)
    dy = _randn(B, T, C, seed=73)
    grads = []
    for _ in range(2):
        wte = torch.nn.Parameter(_randn(V, C, seed=74))
        wpe = torch.nn.Parameter(_randn(T, C, seed=75))
        wte.grad = torch.full((V, C), 0.5, device=DEV, dtype=torch.bfloat16)
        wpe.grad = torch.full((T, C), -0.25, device=DEV, dtype=torch.bfloat16)
        fired = []
        for p in (wte, wpe):
            p._dlbb_grad_sink = fired.append
        wte._dlbb_sink_uses = 2            # tied: ready only after a second use
        embedding(idx, wte, wpe).backward(dy)
        assert len(fired) == 1 and fired[0] is wpe   # wte has one use left
        grads.append((wte.grad.clone(), wpe.grad.clone()))
    ref_e = torch.zeros(V, C, device=DEV).index_add_(0, idx.reshape(-1),
                                                     dy.float().reshape(-1, C)) + 0.5
    ref_p = dy.float().sum(0) - 0.25
    torch.testing.assert_close(grads[0][0].float(), ref_e, rtol=1e-2, atol=3e-2)
    torch.testing.assert_close(grads[0][1].float(), ref_p, rtol=1e-2, atol=3e-2)
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


def test_gemm_autotune_beside_comm_keeps_to_hand_written_kernels(monkeypatch):
    """Inside ``gemm.concurrent_comm()`` (the overlapped TP forward) a shape is tuned under its
    own key and only among the non-persistent hand-written kernels: hipBLASLt's persistent
    Stream-K grids stall when comm workgroups hold CUs."""
    from distributed_llm_backend_benchmark_amd.ops import gemm, linear

    monkeypatch.setenv("DLBB_GEMM", "auto")
    x = _randn(1024, 512, seed=3, scale=0.5)
    w = _randn(768, 512, seed=4, scale=0.5)
    with gemm.concurrent_comm():
        y = linear(x, w, out_dtype=torch.float32)
    keys = [k for k in gemm.CHOICES if k[:3] == (1024, 768, 512) and k[-1] == "concurrent"]
    assert keys and all(gemm.CHOICES[k] == "mfma" for k in keys), gemm.CHOICES
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(y, ref, rtol=2e-3, atol=2e-3 * 512 ** 0.5)
    assert gemm._CONCURRENT[0] == 0


@pytest.mark.parametrize("M,N,K", [(4096, 1536, 4096), (4096, 2048, 4096), (4096, 3072, 1024),
                                   (1000, 640, 1024), (520, 384, 2048), (2048, 1024, 512)])
@pytest.mark.parametrize("epi", ["plain_f32", "bias_gelu_pre_res", "plain_bf16"])
def test_gemm_nt_streamk_matches_fp32(M, N, K, epi):
    """Stream-K NT ping-pong (equal K-tile ranges per CU, split tiles combined in the launch by
    the last-arriving wave) for grids below one round of the CUs, against fp32: ragged M, tiles
    split between 2-4 ranges, the whole epilogue chain; run twice so the arrival counters are
    shown to be left zero."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    x = _randn(M, K, seed=51, scale=0.3)
    w = _randn(N, K, seed=52, scale=0.3)
    b = _randn(N, seed=53)
    r = _randn(M, N, seed=54)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    plan = gemm.streamk_plan(M, N, K, ncu)
    assert plan is not None and gemm.streamk_ok(x, w), plan
    u = x.float() @ w.float().t()
    for _ in range(2):
        if epi == "plain_f32":
            y = torch.empty(M, N, dtype=torch.float32, device=DEV)
            gemm._mfma_streamk_linear(x, w, None, None, None, y, None)
            torch.testing.assert_close(y, u, rtol=2e-3, atol=2e-3 * K ** 0.5)
        elif epi == "plain_bf16":
            y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm._mfma_streamk_linear(x, w, None, None, None, y, None)
            torch.testing.assert_close(y.float(), u, rtol=2e-2, atol=2e-2 * K ** 0.5)
        else:
            y = torch.empty(M, N, dtype=torch.float32, device=DEV)
            pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            gemm._mfma_streamk_linear(x, w, b, "gelu", r, y, pre)
            ub = u + b.float()
            torch.testing.assert_close(y, F.gelu(ub) + r.float(), rtol=2e-3, atol=2e-3 * K ** 0.5)
            torch.testing.assert_close(pre.float(), ub, rtol=2e-2, atol=2e-2 * K ** 0.5)
        torch.cuda.synchronize()
    _, cnt = gemm._SK_WS[(0, _lib_stream())]
    assert int(cnt.abs().sum()) == 0


def _lib_stream():
    from distributed_llm_backend_benchmark_amd.ops import _lib

    return _lib.stream(torch.device(DEV))


def test_gemm_nt_streamk_repeatable():
    """Repeated launches agree to fp32 rounding: the last-arriving wave of a split tile adds the
    other contributors' blocks to its own, so the summation order follows the arrival order
    (like float-atomic split-K), never more than one rounding per contributor apart."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    M, N, K = 4096, 1536, 4096
    x = _randn(M, K, seed=61, scale=0.3)
    w = _randn(N, K, seed=62, scale=0.3)
    ys = []
    for _ in range(3):
        y = torch.empty(M, N, dtype=torch.float32, device=DEV)
        gemm._mfma_streamk_linear(x, w, None, None, None, y, None)
        ys.append(y)
    torch.cuda.synchronize()
    for y in ys[1:]:
        torch.testing.assert_close(y, ys[0], rtol=1e-5, atol=1e-4)


def test_gemm_autotune_offers_tile_variants(monkeypatch):
    """The linear autotuner times the 256 x 192, Stream-K and split-K candidates where their
    contracts hold, and records whichever it picks."""
    from distributed_llm_backend_benchmark_amd.ops import gemm, linear

    monkeypatch.setenv("DLBB_GEMM", "auto")
    x = _randn(4096, 4096, seed=61, scale=0.3)
    w = _randn(1536, 4096, seed=62, scale=0.3)
    y = linear(x, w)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), rtol=2e-2, atol=1.5)
    kind, key, times, best = gemm.TUNE_LOG[-1]
    assert set(times) == {"mfma", "mfma192", "mfma192p", "mfma_sk", "mfma_split", "blas"}, times
    assert gemm.CHOICES[key] == best


@pytest.mark.parametrize("M,N,K", [(4096, 9600, 768), (2000, 19200, 640), (1040, 1536, 1024),
                                   (16384, 3840, 384)])
@pytest.mark.parametrize("bal", [0, 1])
def test_gemm_nt_192_spread_matches_fp32(M, N, K, bal):
    """Persistent 256 x 192 NT GEMM with the C stores spread under the next tile's K-loop
    (variant 2): multi-round grids (several tiles per workgroup), ragged M, the shortest
    reduction it accepts (6 K-tiles) and both DMA schedules — against
    fp32, and bit-identical to the non-persistent 256 x 192 kernel (same MFMA order)."""
    from distributed_llm_backend_benchmark_amd.ops import _lib, gemm

    lib = _lib.lib()
    x = _randn(M, K, seed=71, scale=0.3)
    w = _randn(N, K, seed=72, scale=0.3)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    y1 = torch.empty_like(y)
    try:
        lib.dlbb_gemm_set_bal(bal)
        y.fill_(7.0)
        gemm._mfma192p_linear(x, w, None, None, None, y, None)
        gemm._mfma192_linear(x, w, None, None, None, y1, None)
        torch.cuda.synchronize()
    finally:
        lib.dlbb_gemm_set_bal(2)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), rtol=2e-2,
                               atol=2e-2 * K ** 0.5)
    assert torch.equal(y, y1)


@pytest.mark.parametrize("split", [1, 3, 7, 9, 16, 19])
@pytest.mark.parametrize("dt_out", ["bf16", "fp32"])
def test_split_reduce_matches_fp32(split, dt_out):
    """The weight-gradient split-K reduce (all slabs in flight, streaming loads; templated splits
    and the runtime-split fallback) against an fp32 sum of the slabs, accumulating into an
    existing output, with the bias slabs."""
    from distributed_llm_backend_benchmark_amd.ops import _lib

    N, K = 384, 256
    n, nb = N * K, N
    g = torch.Generator(device=DEV).manual_seed(split)
    ws = torch.randn(split * (n + nb), device=DEV, generator=g)
    dt = torch.bfloat16 if dt_out == "bf16" else torch.float32
    o = torch.randn(n, device=DEV, generator=g).to(dt)
    ob = torch.randn(nb, device=DEV, generator=g).to(dt)
    ref = ws[:split * n].view(split, n).sum(0) + o.float()
    refb = ws[split * n:].view(split, nb).sum(0) + ob.float()
    _lib.check(_lib.lib().dlbb_split_reduce(ws.data_ptr(), o.data_ptr(),
                                            1 if dt_out == "bf16" else 0, n, ob.data_ptr(),
                                            nb, split, 1, _lib.stream(ws.device)),
               "split_reduce")
    torch.cuda.synchronize()
    tol = dict(rtol=1e-2, atol=1e-2) if dt_out == "bf16" else dict(rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(o.float(), ref, **tol)
    torch.testing.assert_close(ob.float(), refb, **tol)


@pytest.mark.parametrize("n,vocab", [(1, 10), (1000, 50304), (16384, 50304), (16384, 7),
                                     (5000, 262144), (16383, 2)])
def test_sort_ids_matches_stable_torch_sort(n, vocab):
    """The one-workgroup id sort of the embedding backward equals torch.sort(stable=True) —
    values AND positions (stability: equal ids keep their order)."""
    from distributed_llm_backend_benchmark_amd.ops.embedding import sort_ids

    g = torch.Generator(device=DEV).manual_seed(n)
    ids = torch.randint(0, vocab, (n,), device=DEV, generator=g)
    s, o = sort_ids(ids, vocab)
    rs, ro = torch.sort(ids, stable=True)
    assert torch.equal(s, rs) and torch.equal(o, ro)
