"""Diagnostic: per-parameter error of the DDP-reduced gradient (2 ranks sharing one GPU, gloo
PG) against a full-batch single-process reference, for the process-group all-reduce and the
custom registered kernel, with and without gradient sinks."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from mp_utils import run_multiprocess  # noqa: E402


def worker(rank, world):
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    comm = init_distributed("gloo", device="cuda")
    cfg = GPT2Config(vocab_size=512, block_size=64, n_layer=2, n_head=4, n_embd=256)
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 512, (world * 2, 65), generator=g).cuda()
    local = data[rank * 2:(rank + 1) * 2]
    ref = GPT2(cfg, device=torch.device("cuda"), seed=3)
    ref(data[:, :-1], data[:, 1:]).backward()
    refg = {n: p.grad.float() for n, p in ref.named_parameters()}
    out = {}
    for tag, ar, sinks, world_pg in (("pg", "rccl", True, True), ("pg_nosink", "rccl", False, True),
                                     ("car", "custom", True, True), ("local", "rccl", True, False)):
        m = GPT2(cfg, device=torch.device("cuda"), seed=3)
        if not sinks:
            for p in m.parameters():
                p._dlbb_single_use = False
        tr = FlatParamTrainer(m, comm if world_pg else None, lr=1e-3, bucket_mb=0.5,
                              allreduce=ar)
        tr.zero_grad()
        tr._reset()
        m(local[:, :-1], local[:, 1:]).backward()
        tr.finish()
        torch.cuda.synchronize()
        errs = []
        for n, p in m.named_parameters():
            o = tr._offsets[id(p)]
            gg = tr.flat_grad[o:o + p.numel()].float().view_as(p) / (world if world_pg else 1)
            if not world_pg:
                continue
            e = float((gg - refg[n]).abs().max()) / max(1e-6, float(refg[n].abs().max()))
            errs.append((round(e, 4), n))
        errs.sort(reverse=True)
        out[tag] = errs[:4]
        tr.close()
    comm.destroy()
    return out


if __name__ == "__main__":
    for r in run_multiprocess(worker, 2, timeout=300):
        for k, v in r.items():
            print(k, v)
