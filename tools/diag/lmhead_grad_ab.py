"""Diagnostic: one GPT-2 forward + backward (fixed weights, fixed batch) with the LM-head forward
GEMM pinned to our kernel vs hipBLASLt (everything else identical): per-parameter relative
gradient difference, then 12 training steps of each (losses)."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from distributed_llm_backend_benchmark_amd.models import gpt2 as G  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops import gemm  # noqa: E402
from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer  # noqa: E402

cfg = G.GPT2Config()
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
idx = torch.randint(0, cfg.vocab_size, (16, 1025), device=dev, generator=g)


def pin(choice):
    for k in list(gemm.CHOICES):
        if k[1] == cfg.vocab_size:
            gemm.CHOICES[k] = choice


grads = {}
for choice in ("mfma", "blas"):
    m = G.GPT2(cfg, device=dev, seed=5)
    loss = m(idx[:, :-1], idx[:, 1:])          # tunes on first use
    pin(choice)
    m.zero_grad(set_to_none=True)
    loss = m(idx[:, :-1], idx[:, 1:])
    loss.backward()
    grads[choice] = (float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()})
print("loss", grads["mfma"][0], grads["blas"][0])
worst = []
for n in grads["mfma"][1]:
    a, b = grads["mfma"][1][n], grads["blas"][1][n]
    rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
    worst.append((rel, n))
worst.sort(reverse=True)
print("largest per-parameter rel grad diff:", [(n, round(r, 5)) for r, n in worst[:8]])
for choice in ("mfma", "blas"):
    m = G.GPT2(cfg, device=dev, seed=5)
    tr = FlatParamTrainer(m, None, lr=3e-4)
    m(idx[:, :-1], idx[:, 1:])
    pin(choice)
    ls = [round(tr.step(idx[:, :-1], idx[:, 1:]), 4) for _ in range(12)]
    print(choice, ls, flush=True)
    tr.close()
