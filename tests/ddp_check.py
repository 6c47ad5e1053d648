"""DDP equivalence worker shared by the ranks-on-one-GPU rehearsal (gloo process group over GPU
tensors, ``test_comm_gpu.py``) and the one-process-per-GPU integration test
(``test_multigpu_integration.py``): the reference's only data-parallel step
(``test/ds_mpi_test.py:27-49``, ``test/ccl.py:92-115``) made checkable.

After one overlapped step the all-reduced gradient must equal a world-1 run on the concatenated
global batch (bf16 tolerance; fp32 buckets tighter), and after a few optimizer steps every rank
must hold bitwise-identical parameters."""

import hashlib
import os


def ddp_equivalence_worker(rank, world, backend, allreduce, fp32_buckets):
    import torch

    if backend == "rccl":
        os.environ["LOCAL_RANK"] = str(rank)
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    comm = init_distributed(backend, device="cuda" if backend == "gloo" else None)
    comm.install_tune_agreement()
    dev = comm.device
    cfg = GPT2Config(vocab_size=512, block_size=64, n_layer=2, n_head=4, n_embd=256)
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 512, (world * 2, 65), generator=g).to(dev)
    local = data[rank * 2:(rank + 1) * 2]

    # world-1 reference on the whole global batch (same seed: same initial weights everywhere)
    ref = GPT2(cfg, device=dev, seed=3)
    loss = ref(data[:, :-1], data[:, 1:])
    loss.backward()
    ref_grads = {n: p.grad.float().clone() for n, p in ref.named_parameters()}
    del ref

    m = GPT2(cfg, device=dev, seed=3)
    kw = dict(mode="flatten", grad_dtype=torch.float32) if fp32_buckets else {}
    tr = FlatParamTrainer(m, comm, lr=1e-3, bucket_mb=0.5, allreduce=allreduce, **kw)
    tr.zero_grad()
    tr._reset()
    m(local[:, :-1], local[:, 1:]).backward()
    tr.finish()
    torch.cuda.synchronize()
    worst = 0.0
    for n, p in m.named_parameters():
        o = tr._offsets[id(p)]
        got = tr.flat_grad[o:o + p.numel()].float().view_as(p) / world   # sum -> mean
        want = ref_grads[n]
        worst = max(worst, float((got - want).abs().max()) / max(float(want.abs().max()), 1e-12))
    for _ in range(3):
        tr.step(local[:, :-1], local[:, 1:])
    torch.cuda.synchronize()
    digest = hashlib.sha256(tr.flat_param.view(torch.int16).cpu().numpy().tobytes()).hexdigest()
    digests = comm.all_gather_object(digest)
    nbuckets = len(tr.buckets)
    tr.check_comm_errors()
    tr.close()
    comm.barrier()
    comm.destroy()
    return worst, digests, nbuckets
