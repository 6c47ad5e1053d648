"""Single-GPU virtual-rank harness of the IPC collective kernels (parallel/virtual_ranks.py):
every kernel of csrc/custom_allreduce.hip runs its production device code for W = 2, 4, 8 ranks
in one fused launch and is compared against an fp32 PyTorch reference of the same collective."""

import pytest
import torch

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16


def _vr():
    from distributed_llm_backend_benchmark_amd.parallel import virtual_ranks as vr

    return vr


def _inputs(W, n, seed, dtype=BF16):
    out = []
    for r in range(W):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed + r)
        out.append(torch.randn(n, generator=g, device="cuda").to(dtype))
    return out


def _ok(got, exp, W):
    return torch.allclose(got.float(), exp.float(), rtol=2e-2, atol=5e-2 * W)


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("dtype", [BF16, torch.float32])
def test_allreduce_oneshot_twoshot(W, dtype):
    vr = _vr()
    V = vr.VirtualRanks(W, capacity_bytes=8 << 20)
    try:
        for n in (W * 8 * 3, 4096, 1 << 18):
            xs = _inputs(W, n, 100 + n, dtype)
            ref = sum(x.float() for x in xs)
            for algo in (vr.K_ONESHOT, vr.K_TWOSHOT):
                for _ in range(3):                # epochs cycle through both buffer halves
                    outs = [torch.empty_like(x) for x in xs]
                    V.all_reduce(xs, outs, algo=algo, nblocks=min(16, V.max_blocks(algo, dtype)))
                    torch.cuda.synchronize()
                    assert V.errors() == [0] * W
                    for o in outs:
                        assert _ok(o, ref, W), (W, n, algo)
    finally:
        V.close()


@pytest.mark.parametrize("W", [2, 4, 8])
def test_registered_pull_push_interleaved(W):
    """Registered in-place two-shot (pull and push) interleaved with staged two-shot calls, so
    every staging half is re-read after local writes of another form."""
    vr = _vr()
    V = vr.VirtualRanks(W, capacity_bytes=4 << 20)
    try:
        n = W * 8 * 1000
        bufs = [torch.empty(n, dtype=BF16, device="cuda") for _ in range(W)]
        rid = V.register(bufs)
        for it in range(6):
            xs = _inputs(W, n, 7 * it)
            ref = sum(x.float() for x in xs)
            for b, x in zip(bufs, xs):
                b.copy_(x)
            V.all_reduce_registered(bufs, rid, nblocks=8, push=bool(it % 2))
            outs = [torch.empty_like(x) for x in xs]
            V.all_reduce(xs, outs, algo=vr.K_TWOSHOT, nblocks=8)
            torch.cuda.synchronize()
            assert V.errors() == [0] * W
            for b, o in zip(bufs, outs):
                assert _ok(b, ref, W), (W, it)
                assert _ok(o, ref, W), (W, it)
    finally:
        V.close()


@pytest.mark.parametrize("W", [2, 4, 8])
def test_direct_allgather_reducescatter_alltoall(W):
    vr = _vr()
    V = vr.VirtualRanks(W, capacity_bytes=1 << 20)
    try:
        n = W * 8 * 512
        xs = _inputs(W, n, 55)
        rid = V.register(xs)
        ag = [torch.zeros(W * n, dtype=BF16, device="cuda") for _ in range(W)]
        V.direct(vr.K_AG, xs, rid, ag, nblocks=16)
        rs = [torch.zeros(n // W, dtype=BF16, device="cuda") for _ in range(W)]
        V.direct(vr.K_RS, xs, rid, rs, nblocks=16)
        a2a = [torch.zeros(n, dtype=BF16, device="cuda") for _ in range(W)]
        V.direct(vr.K_A2A, xs, rid, a2a, nblocks=16)
        torch.cuda.synchronize()
        assert V.errors() == [0] * W
        cat = torch.cat(xs)
        tot = sum(x.float() for x in xs).chunk(W)
        c = n // W
        for r in range(W):
            assert torch.equal(ag[r], cat)
            assert _ok(rs[r], tot[r], W)
            assert torch.equal(a2a[r], torch.cat([x[r * c:(r + 1) * c] for x in xs]))
    finally:
        V.close()


def test_oversized_fused_grid_is_refused():
    vr = _vr()
    V = vr.VirtualRanks(8, capacity_bytes=1 << 20)
    try:
        cap = V.max_blocks(vr.K_TWOSHOT)
        assert 1 <= cap <= 256
        if cap < 256:
            xs = _inputs(8, 8 * 8 * 64, 3)
            outs = [torch.empty_like(x) for x in xs]
            with pytest.raises(ValueError, match="resident capacity"):
                V.all_reduce(xs, outs, algo=vr.K_TWOSHOT, nblocks=cap + 1)
    finally:
        V.close()


def test_bad_sizes_rejected_on_host():
    vr = _vr()
    from distributed_llm_backend_benchmark_amd.ops._lib import KernelError

    V = vr.VirtualRanks(4, capacity_bytes=1 << 16)
    try:
        xs = _inputs(4, 8 * 3, 1)                   # not a multiple of 8 x world: no two-shot
        outs = [torch.empty_like(x) for x in xs]
        with pytest.raises(KernelError):
            V.all_reduce(xs, outs, algo=vr.K_TWOSHOT, nblocks=1)
        big = _inputs(4, 1 << 16, 1)                 # 128 KiB > capacity
        with pytest.raises(KernelError):
            V.all_reduce(big, [torch.empty_like(x) for x in big], algo=vr.K_ONESHOT)
    finally:
        V.close()


def test_missing_peer_wait_is_bounded_and_fails_fast():
    """Rank 0 of two enters a one-shot all-reduce alone: its wait ends at the wall-clock bound
    (not a poll count), flags the error, and a second call on the flagged rank skips its waits."""
    import time

    from distributed_llm_backend_benchmark_amd.parallel import custom_allreduce as car

    vr = _vr()      # dtype 1 = bf16 (ops._lib.DT_BF16)
    V = vr.VirtualRanks(2, capacity_bytes=1 << 20)
    car.set_timeout_ms(200)
    try:
        x = torch.ones(4096, device="cuda", dtype=BF16)
        y = torch.empty_like(x)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        V.lib.dlbb_car_allreduce(V.states[0], x.data_ptr(), y.data_ptr(), x.numel(), 1,
                                 vr.K_ONESHOT, 1, s.cuda_stream)
        s.synchronize()
        first = time.perf_counter() - t0
        t0 = time.perf_counter()
        V.lib.dlbb_car_allreduce(V.states[0], x.data_ptr(), y.data_ptr(), x.numel(), 1,
                                 vr.K_ONESHOT, 1, s.cuda_stream)
        s.synchronize()
        second = time.perf_counter() - t0
        assert 0.15 < first < 5.0, first
        assert second < 0.1, second
        assert V.errors() == [1, 0]
    finally:
        car.set_timeout_ms(60000)
        V.close()
