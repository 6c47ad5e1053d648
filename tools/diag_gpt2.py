"""Compare GPT-2 training trajectories: HIP kernels vs torch reference ops (same init/data)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer  # noqa: E402


def traj(kern, lr, steps=8):
    os.environ["DLBB_KERNELS"] = kern
    cfg = GPT2Config(vocab_size=1024, block_size=256, n_layer=2, n_head=4, n_embd=256)
    m = GPT2(cfg, device=torch.device("cuda"))
    tr = FlatParamTrainer(m, None, lr=lr, bucket_mb=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    idx = torch.randint(0, cfg.vocab_size, (4, 256), device="cuda", generator=g)
    return [round(tr.step(idx, idx), 3) for _ in range(steps)]


def grads(kern):
    os.environ["DLBB_KERNELS"] = kern
    cfg = GPT2Config(vocab_size=1024, block_size=256, n_layer=2, n_head=4, n_embd=256)
    m = GPT2(cfg, device=torch.device("cuda"))
    g = torch.Generator(device="cuda").manual_seed(0)
    idx = torch.randint(0, cfg.vocab_size, (4, 256), device="cuda", generator=g)
    loss = m(idx, idx)
    loss.backward()
    return float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()}


for lr in (3e-3, 1e-3):
    print("lr", lr, "hip  ", traj("hip", lr))
    print("lr", lr, "torch", traj("torch", lr))
lh, gh = grads("hip")
lt, gt = grads("torch")
print("loss hip", lh, "torch", lt)
for n in gh:
    a, b = gh[n], gt[n]
    rel = float((a - b).norm() / (b.norm() + 1e-12))
    print(f"{n:32s} rel_err {rel:.4f} |g| {float(b.norm()):.4e}")
