"""Microbenchmarks of the gfx950 kernels vs their torch/hipBLASLt equivalents (device time via
HIP events, median of N). Prints one JSON line per case; used to fill profiles/kernels.md."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd import ops  # noqa: E402


def t_med(fn, iters=20, warm=3, batch=1):
    """Median seconds per call; ``batch`` calls back to back per event pair (steady clocks for
    short memory-bound kernels, as they run inside a collective's staging)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(batch):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e-3 / batch)
    ts.sort()
    return ts[len(ts) // 2]


def rnd(*s, dt=torch.bfloat16):
    return torch.randn(*s, device="cuda").to(dt)


def out(**kw):
    print(json.dumps(kw), flush=True)


which = sys.argv[1:] or ["gemm", "mem"]
if "gemm" in which:
    shapes = [("7B_qkv_P1", 4096, 12288, 4096), ("7B_out_P1", 4096, 4096, 4096),
              ("7B_up_P1", 4096, 16384, 4096), ("7B_down_P1", 4096, 4096, 16384),
              ("7B_up_P8", 4096, 2048, 4096), ("7B_down_P8", 4096, 4096, 2048),
              ("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
              ("gpt2_fc", 16384, 3072, 768), ("gpt2_lmhead", 16384, 50304, 768)]
    for name, M, N, K in shapes:
        x, w = rnd(M, K), rnd(N, K)
        fl = 2.0 * M * N * K
        from distributed_llm_backend_benchmark_amd.ops.gemm import set_stagger, set_tile
        os.environ["DLBB_GEMM"] = "mfma"
        res = {}
        for tile in (128, 256):
            set_tile(tile)
            res[tile] = t_med(lambda: ops.linear(x, w))
        set_stagger(0)
        res["256ls"] = t_med(lambda: ops.linear(x, w))
        set_stagger(1)
        res["256s1"] = t_med(lambda: ops.linear(x, w))
        set_stagger(2)
        set_tile(0)
        os.environ["DLBB_GEMM"] = "auto"
        th = t_med(lambda: ops.linear(x, w))
        tt = t_med(lambda: torch.matmul(x, w.t()))
        tg = t_med(lambda: ops.linear(x, w, act="gelu"))
        tgt = t_med(lambda: F.gelu(torch.matmul(x, w.t())))
        out(kernel="gemm_bf16_nt", case=name, M=M, N=N, K=K, hip_tflops=fl / th / 1e12,
            t128_tflops=fl / res[128] / 1e12, t256_tflops=fl / res[256] / 1e12,
            t256_lockstep_tflops=fl / res["256ls"] / 1e12, t256_stag1_tflops=fl / res["256s1"] / 1e12,
            hipblaslt_tflops=fl / tt / 1e12, hip_us=th * 1e6, hipblaslt_us=tt * 1e6,
            hip_gelu_us=tg * 1e6, torch_matmul_gelu_us=tgt * 1e6)
if "mem" in which:
    n = 1 << 28  # 256M elements
    srcs = [rnd(n // 8) for _ in range(8)]
    for k in (2, 8):
        t = t_med(lambda: ops.reduce_sum(srcs[:k]))
        b = (k + 1) * srcs[0].numel() * 2
        tt = t_med(lambda: torch.stack(srcs[:k]).float().sum(0).to(torch.bfloat16))
        out(kernel="reduce_sum", nsrc=k, bytes=b, hip_TBps=b / t / 1e12, torch_us=tt * 1e6,
            hip_us=t * 1e6)
    x = rnd(n // 4)
    t = t_med(lambda: ops.cast(x, torch.float32))
    tt = t_med(lambda: x.float())
    out(kernel="cast_bf16_fp32", bytes=x.numel() * 6, hip_TBps=x.numel() * 6 / t / 1e12,
        torch_TBps=x.numel() * 6 / tt / 1e12)
    for rows, cols in ((16384, 768), (4096, 4096), (4096, 8192)):
        a, r = rnd(rows, cols), rnd(rows, cols)
        wv, bv = rnd(cols), rnd(cols)
        t = t_med(lambda: ops.layernorm(a, wv, bv, residual=r))
        tt = t_med(lambda: F.layer_norm(a + r, (cols,), wv, bv))
        b = rows * cols * 2 * 4
        out(kernel="add_layernorm_fwd", rows=rows, cols=cols, hip_TBps=b / t / 1e12,
            hip_us=t * 1e6, torch_us=tt * 1e6)
    a = rnd(16384, 3072)
    bb = rnd(3072)
    t = t_med(lambda: ops.bias_gelu(a, bb, "tanh"))
    tt = t_med(lambda: F.gelu(a + bb, approximate="tanh"))
    out(kernel="bias_gelu_fwd", hip_us=t * 1e6, torch_us=tt * 1e6,
        hip_TBps=a.numel() * 4 / t / 1e12)
    p = torch.randn(124_000_000, device="cuda")
    opt = ops.FlatAdamW(p)
    g = rnd(p.numel())
    sh = torch.empty(p.numel(), dtype=torch.bfloat16, device="cuda")
    t = t_med(lambda: opt.step(g, working_bf16=sh))
    b = p.numel() * (4 * 6 + 2 + 2)
    ref = torch.optim.AdamW([torch.nn.Parameter(p.clone())], fused=True)
    ref.param_groups[0]["params"][0].grad = g.float()
    tt = t_med(lambda: ref.step())
    out(kernel="adamw_flat_124M", hip_us=t * 1e6, hip_TBps=b / t / 1e12,
        torch_fused_adamw_us=tt * 1e6)
if "ln" in which:
    # GPT-2 small LayerNorm shapes: rows = B*T = 16384, cols = 768 (bf16 params, fused residual)
    for rows, cols in ((16384, 768), (16384, 1024), (4096, 4096)):
        a, r = rnd(rows, cols), rnd(rows, cols)
        wv, bv = rnd(cols), rnd(cols)
        t_res = t_med(lambda: ops.layernorm(a, wv, bv, residual=r), iters=50)
        t_plain = t_med(lambda: ops.layernorm(a, wv, bv), iters=50)
        ar = a.clone().requires_grad_(True)
        wr, br = wv.clone().requires_grad_(True), bv.clone().requires_grad_(True)
        y, _ = ops.layernorm(ar, wr, br)
        dy = rnd(rows, cols)
        t_bwd = t_med(lambda: torch.autograd.grad(y, [ar, wr, br], dy, retain_graph=True),
                      iters=50)
        out(kernel="layernorm", rows=rows, cols=cols, fwd_res_us=t_res * 1e6,
            fwd_res_TBps=rows * cols * 2 * 4 / t_res / 1e12, fwd_us=t_plain * 1e6,
            bwd_us=t_bwd * 1e6, bwd_TBps=rows * cols * 2 * 3 / t_bwd / 1e12)
if "wgrad" in which:
    from distributed_llm_backend_benchmark_amd.ops.gemm import wgrad
    for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        M = 16384
        dy, x = rnd(M, N), rnd(M, K)
        w_out, b_out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16), \
            torch.empty(N, device="cuda", dtype=torch.bfloat16)
        t_w = t_med(lambda: wgrad(dy, x, out=w_out), iters=30)
        t_wb = t_med(lambda: wgrad(dy, x, out=w_out, bias_out=b_out), iters=30)
        t_sum = t_med(lambda: dy.sum(0, dtype=torch.float32).to(torch.bfloat16), iters=30)
        out(kernel="wgrad", M=M, N=N, K=K, wgrad_us=t_w * 1e6, wgrad_fused_bias_us=t_wb * 1e6,
            torch_colsum_us=t_sum * 1e6, tflops=2 * M * N * K / t_w / 1e12)
if "wgrad256" in which:
    # weight-gradient GEMM at the GPT-2 shapes: 128 x 128 vs 256 x 128 output tiles vs library
    from distributed_llm_backend_benchmark_amd.ops.gemm import _wgrad_blas, _wgrad_hip, _wgrad_hip256
    for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        M = 16384
        dy, x = rnd(M, N), rnd(M, K)
        w_out, b_out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16), \
            torch.empty(N, device="cuda", dtype=torch.bfloat16)
        res = {}
        for name, fn in (("t128", _wgrad_hip), ("t256", _wgrad_hip256), ("blas", _wgrad_blas)):
            res[name] = t_med(lambda: fn(dy, x, w_out, True, None, b_out), iters=30) * 1e6
        if N % 256 == 0:
            for sp in (6, 7, 8, 9):
                res[f"t256_split{sp}"] = t_med(
                    lambda: _wgrad_hip256(dy, x, w_out, True, sp, b_out), iters=30) * 1e6
        out(kernel="wgrad_tiles", M=M, N=N, K=K, us=res,
            tflops={k: round(2 * M * N * K / v / 1e6, 1) for k, v in res.items()})
if "wgradsplit" in which:
    # total weight-gradient time (split-K GEMM + partial reduce, accumulate + fused bias) by
    # split, both tiles: the split heuristic targets the GEMM alone
    from distributed_llm_backend_benchmark_amd.ops.gemm import _wgrad_hip, _wgrad_hip256
    for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        M = 16384
        dy, x = rnd(M, N), rnd(M, K)
        w_out, b_out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16), \
            torch.empty(N, device="cuda", dtype=torch.bfloat16)
        res = {}
        for sp in (None, 1, 2, 3, 4, 6, 8, 12, 16, 24):
            res[f"t128_s{sp}"] = round(t_med(lambda: _wgrad_hip(dy, x, w_out, True, sp, b_out),
                                             iters=30) * 1e6, 1)
            if N % 256 == 0:
                res[f"t256_s{sp}"] = round(t_med(
                    lambda: _wgrad_hip256(dy, x, w_out, True, sp, b_out), iters=30) * 1e6, 1)
        best = min(res, key=res.get)
        out(kernel="wgrad_split_total", M=M, N=N, K=K, best=best, us=res)
if "xent" in which:
    # fused in-place LM-head loss pass (logits -> dlogits + per-row loss), v1 vs v2, at the
    # GPT-2 step shape; the pass is in place, so each timed call first restores the logits
    # from a copy and the copy's own time is subtracted
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    rows, V = 16384, 50304
    src = (rnd(rows, V) * 2).to(torch.bfloat16)
    buf = torch.empty_like(src)
    tgt = torch.randint(0, V, (rows,), device="cuda")
    loss = torch.empty(rows, device="cuda")
    sc = torch.full((1,), 1.0 / rows, device="cuda")
    t_copy = t_med(lambda: buf.copy_(src), iters=20)
    res = {}
    for var in (1, 2):
        L.lib().dlbb_xent_set_variant(var)

        def run():
            buf.copy_(src)
            L.check(L.lib().dlbb_xent_fused(buf.data_ptr(), tgt.data_ptr(), loss.data_ptr(), rows,
                                            V, V, sc.data_ptr(), L.stream(buf.device)), "xent")
        res[var] = t_med(run, iters=20) - t_copy
    L.lib().dlbb_xent_set_variant(2)
    nbytes = rows * V * 2 * 2
    out(kernel="xent_fused", rows=rows, V=V, v1_us=res[1] * 1e6, v2_us=res[2] * 1e6,
        v1_TBps=nbytes / res[1] / 1e12, v2_TBps=nbytes / res[2] / 1e12, copy_us=t_copy * 1e6)
if "gelu" in which:
    a, bb, g = rnd(16384, 3072), rnd(3072), rnd(16384, 3072)
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    du = torch.empty_like(a)
    ws = torch.zeros(3072, dtype=torch.float32, device="cuda")
    t_f = t_med(lambda: ops.bias_gelu(a, bb, "tanh"), iters=30)
    t_b = t_med(lambda: L.lib().dlbb_bias_gelu_bwd(g.data_ptr(), a.data_ptr(), None, du.data_ptr(),
                                                   None, 16384, 3072, 1, L.stream(a.device)), iters=30)
    t_bd = t_med(lambda: L.lib().dlbb_bias_gelu_bwd(g.data_ptr(), a.data_ptr(), None, du.data_ptr(),
                                                    ws.data_ptr(), 16384, 3072, 1, L.stream(a.device)), iters=30)
    out(kernel="bias_gelu_tanh", fwd_us=t_f * 1e6, fwd_TBps=a.numel() * 4 / t_f / 1e12,
        bwd_us=t_b * 1e6, bwd_db_us=t_bd * 1e6, bwd_TBps=a.numel() * 6 / t_b / 1e12)
if "lnab" in which:
    # LayerNorm backward, raw launcher (kernel + dgamma/dbeta column reduce); bytes = h + dy
    # (+ dres) read + dx written
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    for rows, cols in ((16384, 768), (16384, 1024), (4096, 768)):
        h, dy, dres = rnd(rows, cols), rnd(rows, cols), rnd(rows, cols)
        gam = rnd(cols)
        mean = torch.randn(rows, device="cuda")
        rstd = torch.rand(rows, device="cuda") + 0.5
        dx = torch.empty_like(h)
        grid = L.lib().dlbb_layernorm_bwd_grid(rows)
        ws = torch.empty(2 * grid * cols, device="cuda")
        dg, db = torch.empty(cols, device="cuda", dtype=torch.bfloat16), \
            torch.empty(cols, device="cuda", dtype=torch.bfloat16)
        res = {}
        for var in (0,):
            for with_res in (False, True):
                def run():
                    L.check(L.lib().dlbb_layernorm_bwd(
                        dy.data_ptr(), h.data_ptr(), gam.data_ptr(), 1, mean.data_ptr(),
                        rstd.data_ptr(), dres.data_ptr() if with_res else None, dx.data_ptr(),
                        ws.data_ptr(), dg.data_ptr(), db.data_ptr(), rows, cols, 0,
                        L.stream(h.device)), "ln_bwd")
                t = t_med(run, iters=50)
                nb = rows * cols * 2 * (4 if with_res else 3)
                res[f"{'res' if with_res else 'nores'}"] = {
                    "us": round(t * 1e6, 2), "TBps": round(nb / t / 1e12, 3)}
        out(kernel="layernorm_bwd", rows=rows, cols=cols, res=res)
if "wgradfused" in which:
    # weight gradient at the GPT-2 shapes: separate split-K reduce pass vs in-launch combine
    # (both workgroup orders), accumulate into bf16 + fused bias (the training-step call)
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    from distributed_llm_backend_benchmark_amd.ops import gemm as G
    from distributed_llm_backend_benchmark_amd.ops.gemm import (_wgrad_hip, _wgrad_hip256,
                                                                _wgrad_hip_wide)
    for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        M = 16384
        dy, x = rnd(M, N), rnd(M, K)
        w_out = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        b_out = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        res = {}
        for name, fn in (("t128", _wgrad_hip), ("t256", _wgrad_hip256), ("wide", _wgrad_hip_wide)):
            if name == "t256" and N % 256 or name == "wide" and K % 256:
                continue
            for mode in ("sep", "fused_split_major", "fused_tile_major"):
                G.set_wgrad_fused(mode != "sep")
                L.lib().dlbb_gemm_wgrad_set_order(1 if mode == "fused_tile_major" else 0)
                res[f"{name}_{mode}"] = round(t_med(
                    lambda: fn(dy, x, w_out, True, None, b_out), iters=30) * 1e6, 1)
        G.set_wgrad_fused(False)
        L.lib().dlbb_gemm_wgrad_set_order(1)
        out(kernel="wgrad_fused_reduce_ab", M=M, N=N, K=K, us=res,
            tflops={k: round(2 * M * N * K / v / 1e6, 1) for k, v in res.items()})
if "memroof" in which:
    # collective-path memory kernels against the HBM roofline:
    # cast (every dtype pair) vs torch's copy, strided pack, chunk-copy flatten / list unpack,
    # chunk-copy with scale, n-way reduce — 64 MiB .. 1 GiB of source
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    from distributed_llm_backend_benchmark_amd.ops.elementwise import ChunkTable, ScaleTable
    dts = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}
    for mib in (64, 256, 1024):
        MB = 10 if mib <= 256 else 4
        for si, so in (("bf16", "fp32"), ("fp32", "bf16"), ("fp16", "fp32"), ("fp32", "fp16"),
                       ("bf16", "fp16"), ("bf16", "bf16"), ("fp32", "fp32")):
            n = (mib << 20) // dts[si].itemsize
            x = rnd(n, dt=dts[si])
            y = torch.empty(n, device="cuda", dtype=dts[so])
            nb = n * (dts[si].itemsize + dts[so].itemsize)
            res = {"ours": t_med(lambda: ops.cast(x, dts[so], out=y), iters=15, batch=MB)}
            tt = t_med(lambda: y.copy_(x), iters=15, batch=MB)
            out(kernel="cast", src=si, dst=so, src_MiB=mib,
                TBps={k: round(nb / v / 1e12, 3) for k, v in res.items()},
                torch_copy_TBps=round(nb / tt / 1e12, 3))
        # strided pack: the QKV column slice [rows, 3H] -> [rows, H] bf16
        cols = 4096
        rows = (mib << 20) // (2 * cols)
        src = rnd(rows, 3 * cols)
        dst = torch.empty(rows, cols, device="cuda", dtype=torch.bfloat16)
        t = t_med(lambda: ops.pack_rows(src[:, :cols], out=dst), iters=15, batch=MB)
        tt = t_med(lambda: dst.copy_(src[:, :cols]), iters=15, batch=MB)
        nb = rows * cols * 4
        out(kernel="pack_rows", src_MiB=mib, TBps=round(nb / t / 1e12, 3),
            torch_copy_TBps=round(nb / tt / 1e12, 3))
        # chunk-copy: the list unpack of an 8-rank all-gather (8 equal slices -> 8 tensors)
        n = (mib << 20) // 2
        flat = rnd(n)
        outs = [torch.empty(n // 8, device="cuda", dtype=torch.bfloat16) for _ in range(8)]
        tab = ChunkTable([(flat[i * (n // 8):(i + 1) * (n // 8)], outs[i]) for i in range(8)])
        L.lib().dlbb_chunk_copy_set_nt(0)
        t = t_med(tab.run, iters=15, batch=MB)
        L.lib().dlbb_chunk_copy_set_nt(1)
        tnt = t_med(tab.run, iters=15, batch=MB)
        L.lib().dlbb_chunk_copy_set_nt(2)
        tauto = t_med(tab.run, iters=15, batch=MB)
        tt = t_med(lambda: [o.copy_(flat[i * (n // 8):(i + 1) * (n // 8)])
                            for i, o in enumerate(outs)], iters=15, batch=MB)
        out(kernel="chunk_copy", src_MiB=mib, chunks=tab.nchunks,
            TBps=round(2 * n * 2 / t / 1e12, 3), nt_TBps=round(2 * n * 2 / tnt / 1e12, 3),
            auto_TBps=round(2 * n * 2 / tauto / 1e12, 3),
            torch_8copies_TBps=round(2 * n * 2 / tt / 1e12, 3))
        g32 = torch.empty(n, device="cuda")
        st = ScaleTable([(flat, g32)], 0.125)
        t = t_med(st.run, iters=15, batch=MB)
        out(kernel="chunk_copy_scale_bf16_fp32", src_MiB=mib, TBps=round(n * 6 / t / 1e12, 3))
        srcs = [rnd(n // 8) for _ in range(8)]
        t = t_med(lambda: ops.reduce_sum(srcs), iters=15, batch=MB)
        out(kernel="reduce_sum_8src", src_MiB=mib, TBps=round(9 * (n // 8) * 2 / t / 1e12, 3))
if "splitred" in which:
    # the weight-gradient split-K reduce alone (fp32 slabs -> bf16 dW += sum, + bias slabs; all
    # slabs in flight, non-temporal loads) at the GPT-2 dW shapes and the splits the step uses; bytes = slabs read + dW read + written
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    for N, K, splits in ((2304, 768, (8, 9)), (768, 768, (6, 16)), (3072, 768, (6, 7, 9)),
                         (768, 3072, (6, 7))):
        n, nb = N * K, N
        for sp in splits:
            ws = torch.randn(sp * (n + nb), device="cuda")
            o = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
            ob = torch.zeros(nb, device="cuda", dtype=torch.bfloat16)
            res = {}
            for var in (0,):
                t = t_med(lambda: L.check(L.lib().dlbb_split_reduce(
                    ws.data_ptr(), o.data_ptr(), 1, n, ob.data_ptr(), nb, sp, 1,
                    L.stream(ws.device)), "split_reduce"), iters=50)
                nbytes = sp * (n + nb) * 4 + 2 * (n + nb) * 2
                res = {"us": round(t * 1e6, 2), "TBps": round(nbytes / t / 1e12, 3)}
            out(kernel="split_reduce", N=N, K=K, split=sp, res=res)
if "wgradpp" in which:
    # GPT-2 dW shapes on the 256^2 ping-pong TN kernel with split-K over all tokens (fp32 slabs
    # + the NN split reduce), vs the tuned default (128 x 256 / 256 x 128 wgrad tiles with the
    # fused bias); the bias column sum the TN path would need is timed on its own
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    from distributed_llm_backend_benchmark_amd.ops.gemm import (_pp_launch, _wgrad_hip,
                                                                _wgrad_hip256, _wgrad_hip_wide)
    for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        M = 16384
        dy, x = rnd(M, N), rnd(M, K)
        w_out = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        b_out = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        ref = (dy.float().t() @ x.float())
        res, err = {}, {}
        res["t128_bias"] = round(t_med(lambda: _wgrad_hip(dy, x, w_out, False, None, b_out),
                                       iters=30) * 1e6, 1)
        if N % 256 == 0:
            res["t256x128_bias"] = round(t_med(
                lambda: _wgrad_hip256(dy, x, w_out, False, None, b_out), iters=30) * 1e6, 1)
        if K % 256 == 0:
            res["t128x256_bias"] = round(t_med(
                lambda: _wgrad_hip_wide(dy, x, w_out, False, None, b_out), iters=30) * 1e6, 1)
            res["t128x256_nobias"] = round(t_med(
                lambda: _wgrad_hip_wide(dy, x, w_out, False, None, None), iters=30) * 1e6, 1)
        res["colsum_torch"] = round(t_med(lambda: dy.sum(0, dtype=torch.float32), iters=30)
                                    * 1e6, 1)
        for sp in (1, 2, 3, 4, 6, 8, 9, 12, 16):
            if M // 64 < sp:
                continue
            res[f"pp_s{sp}"] = round(t_med(lambda: _pp_launch(dy, x, w_out, False, 0, N, sp),
                                           iters=30) * 1e6, 1)
            err[f"pp_s{sp}"] = round(float((w_out.float() - ref).abs().max()
                                           / ref.abs().max()), 5)
        fl = 2.0 * M * N * K
        best = min((k for k in res if k != "colsum_torch"), key=res.get)
        out(kernel="wgrad_pp_split", M=M, N=N, K=K, best=best, us=res, rel_err=err,
            tflops={k: round(fl / v / 1e6, 1) for k, v in res.items() if k != "colsum_torch"})


if "wgradstages" in which:
    # weight-gradient LDS ring depth (2 / 3 stages) x split at the GPT-2 dW shapes, whole call
    # (GEMM + reduce, fused bias, accumulate): the asm transposed reads keep the DMA prefetch in
    # flight, so a deeper ring can now pay
    from distributed_llm_backend_benchmark_amd.ops import _lib as L
    from distributed_llm_backend_benchmark_amd.ops.gemm import _wgrad_hip, _wgrad_hip256
    for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        M = 16384
        dy, x = rnd(M, N), rnd(M, K)
        w_out, b_out = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16), \
            torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        res = {}
        for nb in (2, 3):
            L.lib().dlbb_gemm_wgrad_set_stages(nb)
            for sp in (None, 4, 6, 8, 12):
                res[f"t128_nb{nb}_s{sp}"] = round(t_med(
                    lambda: _wgrad_hip(dy, x, w_out, True, sp, b_out), iters=30) * 1e6, 1)
                if N % 256 == 0:
                    res[f"t256_nb{nb}_s{sp}"] = round(t_med(
                        lambda: _wgrad_hip256(dy, x, w_out, True, sp, b_out), iters=30) * 1e6, 1)
        L.lib().dlbb_gemm_wgrad_set_stages(2)
        best = min(res, key=res.get)
        out(kernel="wgrad_stages", M=M, N=N, K=K, best=best, us=res)
