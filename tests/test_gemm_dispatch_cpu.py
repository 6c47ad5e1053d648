"""CPU checks of the GEMM dispatch layer (ops/gemm.py, ops/linear_fn.py) that need no GPU: the
dgrad fallbacks (plain and through a GELU), the NN kernel's split-K heuristic and contract
predicate, and the fused MLP op's CPU path against a float64 autograd reference."""

import pytest
import torch
import torch.nn.functional as F

from distributed_llm_backend_benchmark_amd.ops import gemm
from distributed_llm_backend_benchmark_amd.ops.linear_fn import mlp_train


def test_dgrad_cpu_fallback_plain():
    g = torch.Generator().manual_seed(0)
    dy = torch.randn(64, 96, generator=g).to(torch.bfloat16)
    w = torch.randn(96, 128, generator=g).to(torch.bfloat16)
    out = gemm.dgrad(dy, w)
    torch.testing.assert_close(out.float(), dy.float() @ w.float(), rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("act,approx", [("gelu_tanh", "tanh"), ("gelu", "none")])
def test_dgrad_cpu_fallback_through_gelu(act, approx):
    """dgelu=(u, act) returns (dY @ W) * act'(u): the gradient w.r.t. the pre-activation."""
    g = torch.Generator().manual_seed(1)
    dy = torch.randn(32, 64, generator=g).to(torch.bfloat16)
    w = torch.randn(64, 256, generator=g).to(torch.bfloat16)
    u = (2 * torch.randn(32, 256, generator=g)).to(torch.bfloat16)
    out = gemm.dgrad(dy, w, dgelu=(u, act))
    uf = u.double().requires_grad_(True)
    F.gelu(uf, approximate=approx).backward(dy.double() @ w.double())
    torch.testing.assert_close(out.double(), uf.grad, rtol=2e-2, atol=5e-2)


def test_dgrad_split_heuristic_and_contract():
    # LM-head dX: 192 tiles of 256^2, 786 K-tiles -> split 4 (768 workgroups = 3 rounds)
    assert gemm.dgrad_split(16384, 768, 50304) == 4
    # a full grid or a short reduction: no split
    assert gemm.dgrad_split(16384, 3072, 768) == 1
    assert gemm.dgrad_split(16384, 768, 3072) == 1
    assert gemm.dgrad_split(4096, 4096, 16384) == 1
    bf = torch.bfloat16
    assert gemm.dgrad_supported(torch.empty(64, 128, dtype=bf), torch.empty(128, 256, dtype=bf))
    assert not gemm.dgrad_supported(torch.empty(64, 128, dtype=bf), torch.empty(128, 200, dtype=bf))
    assert not gemm.dgrad_supported(torch.empty(60, 128, dtype=bf), torch.empty(128, 256, dtype=bf))
    assert not gemm.dgrad_supported(torch.empty(64, 100, dtype=bf), torch.empty(100, 256, dtype=bf))


def test_mlp_train_cpu_matches_autograd():
    g = torch.Generator().manual_seed(2)
    x = torch.randn(4, 8, 32, generator=g, dtype=torch.float64, requires_grad=True)
    w1 = (0.1 * torch.randn(128, 32, generator=g, dtype=torch.float64)).requires_grad_(True)
    b1 = (0.1 * torch.randn(128, generator=g, dtype=torch.float64)).requires_grad_(True)
    w2 = (0.1 * torch.randn(32, 128, generator=g, dtype=torch.float64)).requires_grad_(True)
    b2 = (0.1 * torch.randn(32, generator=g, dtype=torch.float64)).requires_grad_(True)
    params = (x, w1, b1, w2, b2)
    y = mlp_train(x, w1, b1, w2, b2, act="gelu_tanh")
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    grads = torch.autograd.grad((y * dy).sum(), params)
    ref = F.linear(F.gelu(F.linear(x, w1, b1), approximate="tanh"), w2, b2)
    ref_grads = torch.autograd.grad((ref * dy).sum(), params)
    torch.testing.assert_close(y, ref)
    for a, b in zip(grads, ref_grads):
        torch.testing.assert_close(a, b)


def test_wgrad_pingpong_contract():
    """TN ping-pong weight gradient: rows N % 128, columns K % 256, tokens % 64, no fused bias,
    accumulate only into bf16; the LM-head and 7B dW shapes qualify."""
    bf = torch.bfloat16

    def ok(T, N, K, acc=False, out_dtype=bf, bias=False):
        dy, x = torch.empty(T, N, dtype=bf), torch.empty(T, K, dtype=bf)
        out = torch.empty(N, K, dtype=out_dtype)
        return gemm.wgrad_pp_supported(dy, x, out, acc, torch.empty(N, dtype=bf) if bias else None)

    assert ok(16384, 50304, 768) and ok(4096, 12288, 4096) and ok(64, 128, 256)
    assert ok(16384, 50304, 768, acc=True)
    assert not ok(16384, 50304, 768, acc=True, out_dtype=torch.float32)
    assert ok(16384, 50304, 768, out_dtype=torch.float32)
    assert ok(16384, 768, 768, bias=True)    # bias gradient: a separate column-sum pass
    assert not ok(16384, 200, 768) and not ok(16384, 768, 640) and not ok(100, 768, 768)
    assert "pp" in gemm._WGRAD_IMPLS


def test_wgrad_pingpong_tail_plan():
    # LM-head dW on 256 CUs: 591 tiles -> 510 in two whole rounds, 81-tile tail split 3 ways
    assert gemm.pp_tail_plan(16384, 50304, 768, 256) == (43520, 3)
    # whole or mostly full last rounds: no tail
    assert gemm.pp_tail_plan(4096, 12288, 4096, 256) == (12288, 1)
    assert gemm.pp_tail_plan(8192, 8192, 8192, 256) == (8192, 1)
    assert gemm.pp_tail_plan(16384, 896, 768, 256) == (896, 1)
    # a large requested split leaves no empty trailing slice (advisor r02: 28 slices of
    # ceil(256/28) = 10 K-tiles would start slices 26, 27 past the 256 K-tiles)
    for shape in [(16384, 44288, 768, 256), (16384, 50304, 768, 256), (4096, 33024, 4096, 256)]:
        head, split = gemm.pp_tail_plan(*shape)
        nkt = shape[0] // 64
        if split > 1:
            kt = -(-nkt // split)
            assert (split - 1) * kt < nkt, (shape, split, kt)


def test_concurrent_comm_switches_off_persistent_forms_in_the_library():
    """inside gemm.concurrent_comm() (GEMMs beside comm kernels) the library's
    persistent GEMM forms (grid = num CUs, all workgroups assumed resident) are off, nested
    contexts included, and back on after."""
    from distributed_llm_backend_benchmark_amd.ops import _lib, gemm

    lib = _lib.lib()
    assert lib.dlbb_gemm_get_concurrent() == 0
    with gemm.concurrent_comm():
        assert lib.dlbb_gemm_get_concurrent() == 1
        with gemm.concurrent_comm():
            assert lib.dlbb_gemm_get_concurrent() == 1
        assert lib.dlbb_gemm_get_concurrent() == 1
    assert lib.dlbb_gemm_get_concurrent() == 0


def test_library_candidate_needs_margin(monkeypatch):
    """The autotuners pick hipBLASLt only when it beats the fastest hand-written candidate by
    more than ``library_margin()`` (host setup cost and co-residency hazards are invisible to
    device-time tuning); DLBB_LIB_MARGIN=0 is plain fastest-wins."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    monkeypatch.delenv("DLBB_LIB_MARGIN", raising=False)
    assert gemm.library_margin() == 0.05
    assert gemm._choose({"mfma": 1.04, "blas": 1.0})[0] == "mfma"
    assert gemm._choose({"mfma": 1.07, "mfma192": 1.049, "blas": 1.0})[0] == "mfma192"
    assert gemm._choose({"mfma": 1.07, "blas": 1.0})[0] == "blas"
    assert gemm._choose({"mfma": 0.9, "blas": 1.0})[0] == "mfma"
    assert gemm._choose({"blas": 1.0})[0] == "blas"
    monkeypatch.setenv("DLBB_LIB_MARGIN", "0")
    assert gemm._choose({"mfma": 1.02, "blas": 1.0})[0] == "blas"
    monkeypatch.setenv("DLBB_LIB_MARGIN", "bogus")
    assert gemm.library_margin() == 0.05
