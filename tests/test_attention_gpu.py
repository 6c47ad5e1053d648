"""Causal flash-attention forward (csrc/attention.hip) vs an fp32 PyTorch reference, and the
fused-QKV autograd path vs torch SDPA autograd."""

import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(qkv, H):
    B, T, C3 = qkv.shape
    C = C3 // 3
    D = C // H
    q, k, v = qkv.float().view(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
    s = q @ k.transpose(-1, -2) / math.sqrt(D)
    mask = torch.ones(T, T, device=qkv.device, dtype=torch.bool).triu(1)
    s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.softmax(s, -1) @ v
    return o.transpose(1, 2).reshape(B, T, C), lse


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("B,T,H", [(2, 64, 3), (2, 200, 2), (1, 256, 4), (2, 1024, 2),
                                   (1, 333, 1)])
def test_attn_fwd_matches_fp32_reference(B, T, H, D):
    """Forward at head dim 64 (GPT-2) and 128 (the TP model's heads) against fp32, incl. T not a
    multiple of the key tile (the clamped last tile)."""
    from distributed_llm_backend_benchmark_amd.ops.attention import attn_fwd

    g = torch.Generator(device="cuda").manual_seed(T + H + D)
    qkv = (torch.randn(B, T, 3 * H * D, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    out, lse = attn_fwd(qkv, H)
    ref, ref_lse = _ref(qkv, H)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse, ref_lse, rtol=1e-3, atol=2e-3)


@pytest.mark.parametrize("D", [64, 128])
def test_attn_fwd_growing_scores(D):
    """Scores whose row max keeps growing along the keys (key rows scaled up with their index):
    every tile rescales the running output."""
    from distributed_llm_backend_benchmark_amd.ops.attention import attn_fwd

    B, T, H = 2, 777, 2
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, T, 3, H, D, device="cuda", generator=g)
    q = torch.randn(D, device="cuda", generator=g) * (64 / D) ** 0.5
    x[:, :, 0] = q + 0.1 * x[:, :, 0]                 # every query ~ q
    ramp = torch.linspace(0.0, 6.0, T, device="cuda").view(1, T, 1, 1)
    x[:, :, 1] = q * ramp + 0.1 * x[:, :, 1]           # scores grow ~ linearly with the key
    qkv = x.reshape(B, T, 3 * H * D).to(torch.bfloat16)
    out, lse = attn_fwd(qkv, H)
    ref, ref_lse = _ref(qkv, H)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse, ref_lse, rtol=1e-3, atol=5e-3)


@pytest.mark.parametrize("D", [64, 128])
def test_attn_asymmetric_values(D):
    """V = one-hot rows: the output picks softmax weights of the right keys (catches a
    transposed V read or a permuted key order in P)."""
    from distributed_llm_backend_benchmark_amd.ops.attention import attn_fwd

    B, T, H = 1, 128, 1
    qkv = torch.zeros(B, T, 3 * H * D, device="cuda")
    qkv[0, :, D:2 * D] = torch.randn(T, D, device="cuda")        # K
    qkv[0, :, :D] = torch.randn(T, D, device="cuda")             # Q
    vv = torch.zeros(T, D, device="cuda")
    vv[torch.arange(T), torch.arange(T) % D] = torch.arange(T, device="cuda").float() / T
    vv[torch.arange(T), (torch.arange(T) * 7 + 3) % D] -= 0.25
    qkv[0, :, 2 * D:] = vv
    qkv = qkv.to(torch.bfloat16)
    out, _ = attn_fwd(qkv, H)
    ref, _ = _ref(qkv, H)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=1e-2)


@pytest.mark.parametrize("D", [64, 128])
def test_causal_attention_autograd_matches_sdpa(D):
    """Fused-QKV autograd path vs torch SDPA (head dim 128: our forward, the stack's backward)."""
    from distributed_llm_backend_benchmark_amd.ops import causal_attention
    from distributed_llm_backend_benchmark_amd.ops.attention import _torch_attention

    B, T, H = 2, 512, 4
    g = torch.Generator(device="cuda").manual_seed(3)
    base = torch.randn(B, T, 3 * H * D, device="cuda", generator=g).to(torch.bfloat16)
    gout = torch.randn(B, T, H * D, device="cuda", generator=g).to(torch.bfloat16)
    x1 = base.clone().requires_grad_(True)
    y1 = causal_attention(x1, H)
    y1.backward(gout)
    x2 = base.clone().requires_grad_(True)
    y2 = _torch_attention(x2, H)
    y2.backward(gout)
    torch.testing.assert_close(y1.float(), y2.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x1.grad.float(), x2.grad.float(), rtol=3e-2, atol=3e-2)


def _ref_grads(qkv, gout, H):
    x = qkv.float().clone().requires_grad_(True)
    y, _ = _ref(x, H)
    y.backward(gout.float())
    return y.detach(), x.grad


@pytest.mark.parametrize("B,T,H", [(1, 64, 1), (2, 200, 2), (1, 256, 3), (2, 1024, 2),
                                   (1, 333, 2)])
def test_attn_bwd_matches_fp32_reference(B, T, H):
    from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd

    g = torch.Generator(device="cuda").manual_seed(7 * T + H)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda", generator=g).to(torch.bfloat16)
    gout = torch.randn(B, T, H * 64, device="cuda", generator=g).to(torch.bfloat16)
    out, lse = attn_fwd(qkv, H)
    d = attn_bwd(qkv, out, lse, gout, H)
    _, ref = _ref_grads(qkv, gout, H)
    C = H * 64
    for j, name in enumerate("qkv"):
        got, want = d[..., j * C:(j + 1) * C].float(), ref[..., j * C:(j + 1) * C]
        err = float((got - want).abs().max())
        scale = float(want.abs().max())
        assert err <= 0.03 * scale + 0.02, (name, err, scale)


def test_workgroup_timeline_stamps():
    """The diagnostic timeline (wg_stamp, tools/attn_timeline.py): with stamp buffers set, every
    workgroup of the three kernels records start <= mid <= end and a CU id, and the outputs are
    bit-identical to an unstamped run; with the buffers cleared nothing is written."""
    from distributed_llm_backend_benchmark_amd.ops import _lib
    from distributed_llm_backend_benchmark_amd.ops.attention import attn_bwd, attn_fwd

    B, T, H = 2, 1024, 4
    g = torch.Generator(device="cuda").manual_seed(3)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda", generator=g).to(torch.bfloat16)
    gout = torch.randn(B, T, H * 64, device="cuda", generator=g).to(torch.bfloat16)
    o0, l0 = attn_fwd(qkv, H)
    d0 = attn_bwd(qkv, o0, l0, gout, H)
    nq = ((T + 127) // 128 + 1) // 2 * H * B
    st = [torch.zeros(nq, 4, dtype=torch.int64, device="cuda") for _ in range(3)]
    L = _lib.lib()
    L.dlbb_attn_set_stamps(st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr())
    try:
        o1, l1 = attn_fwd(qkv, H)
        d1 = attn_bwd(qkv, o1, l1, gout, H)
        torch.cuda.synchronize()
    finally:
        L.dlbb_attn_set_stamps(None, None, None)
    assert torch.equal(o0, o1) and torch.equal(l0, l1) and torch.equal(d0, d1)
    for t in st:
        a = t.cpu()
        assert bool((a[:, 0] > 0).all()) and bool((a[:, 2] >= a[:, 0]).all())
        mid = a[:, 1]
        assert bool(((mid == 0) | ((mid >= a[:, 0]) & (mid <= a[:, 2]))).all())
    before = [t.clone() for t in st]
    attn_fwd(qkv, H)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(st, before))
