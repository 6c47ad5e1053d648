"""Diagnostic: GPT-2 gradients with the fused LM-head loss vs linear + cross_entropy, and a short
training run with each path (loss per step)."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from distributed_llm_backend_benchmark_amd import ops  # noqa: E402
from distributed_llm_backend_benchmark_amd.models import gpt2 as G  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.linear_fn import linear_train  # noqa: E402
from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer  # noqa: E402

fused = ops.linear_cross_entropy


def unfused(x, w, t):
    return ops.cross_entropy(linear_train(x, w), t)


cfg = G.GPT2Config()
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
idx = torch.randint(0, cfg.vocab_size, (16, 1025), device=dev, generator=g)
grads = {}
for name, fn in (("fused", fused), ("unfused", unfused)):
    ops.linear_cross_entropy = fn
    m = G.GPT2(cfg, device=dev, seed=5)
    loss = m(idx[:, :-1], idx[:, 1:])
    loss.backward()
    grads[name] = (float(loss), {n: p.grad.float() for n, p in m.named_parameters()})
for n in ("wte", "wpe", "blocks.0.attn_w", "blocks.11.fc_w", "ln_f.weight"):
    a, b = grads["fused"][1][n], grads["unfused"][1][n]
    print(n, "rel err", float((a - b).abs().max() / b.abs().max()))
print("loss", grads["fused"][0], grads["unfused"][0])
for name, fn in (("fused", fused), ("unfused", unfused)):
    ops.linear_cross_entropy = fn
    m = G.GPT2(cfg, device=dev, seed=5)
    tr = FlatParamTrainer(m, None, lr=3e-4)
    ls = [round(tr.step(idx[:, :-1], idx[:, 1:]), 3) for _ in range(12)]
    print(name, ls)
    tr.close()
