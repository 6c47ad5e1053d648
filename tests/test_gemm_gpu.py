"""Split-K NT GEMM (csrc/gemm.hip dlbb_gemm_bf16_nt_split) against an fp32 PyTorch product."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(4096, 1536, 4096), (4096, 2048, 4096), (1024, 768, 2048),
                                   (520, 384, 1024)])
def test_nt_split_k_matches_fp32(M, N, K):
    """Split-K NT ping-pong (fp32 partials + reduce / cast) against an fp32 product, on the
    TP-7B shard shapes it is tuned for (256 x 192 and 256² tiles) and a ragged M."""
    from distributed_llm_backend_benchmark_amd.ops import gemm

    plan = gemm.split_plan(M, N, K, gemm._num_cus(torch.device("cuda")))
    assert plan is not None
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gemm._mfma_split_linear(x, w, None, None, None, out, None)
    ref = x.float() @ w.float().t()
    err = float((out.float() - ref).abs().max() / ref.abs().max())
    assert err < 1e-2, err
