"""Single-GPU RCCL paths (world 1), the collective sweep engine and the IPC all-reduce protocol
exercised by 2 processes sharing one GPU."""

import json
import os
import subprocess
import sys

import pytest
import torch

from mp_utils import run_multiprocess

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_world1_sweep(tmp_path):
    from distributed_llm_backend_benchmark_amd.bench.sweep import run_1d_sweep, run_3d_sweep
    from distributed_llm_backend_benchmark_amd.parallel.collectives import OPS
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.stats import stats1d, stats3d

    comm = init_distributed("rccl")
    try:
        ops = [o for o in OPS if o != "alltoall_moe"]
        run_1d_sweep(comm, ops=ops, sizes={"1KB": 256, "64KB": 16384}, warmup=2, iters=5,
                     output_dir=str(tmp_path / "r1d"), validate=True, batched=True, graph=True)
        run_3d_sweep(comm, ops=["allreduce", "allgather", "reduce_scatter"], batch_sizes=[1],
                     seq_lengths=[128], hidden_dims=[2048], warmup=2, iters=5,
                     output_dir=str(tmp_path / "r3d"), validate=True, wire_dtype="fp32")
    finally:
        comm.destroy()
    files = sorted(os.listdir(tmp_path / "r1d"))
    errs = [f for f in files if f.endswith(".error.json")]
    assert not errs, [json.load(open(tmp_path / "r1d" / f))["error"] for f in errs]
    for f in files:
        d = json.load(open(tmp_path / "r1d" / f))
        assert d["validated"] is True, f
        assert d["timing_method"] == "hip_event"
        assert len(d["timings"]) == 1 and len(d["timings"][0]) == 5
    rows = stats1d.process_directory(str(tmp_path / "r1d"), str(tmp_path / "s1d"), verbose=False)
    assert len(rows) == len(ops) * 2
    rows3 = stats3d.process_directory(str(tmp_path / "r3d"), str(tmp_path / "s3d"), "rccl",
                                      verbose=False)
    assert {r["wire_dtype"] for r in rows3} == {"float32"}


def test_native_rccl_world1_sweep(tmp_path):
    """Native C++ RCCL engine: every op validated, batched loop captured in a HIP graph, and
    the C++ per-iteration / batched timing loops."""
    from distributed_llm_backend_benchmark_amd.bench.sweep import run_1d_sweep
    from distributed_llm_backend_benchmark_amd.parallel.collectives import make_data
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.rccl_native import NATIVE_OPS, get_native

    comm = init_distributed("rccl")
    try:
        ops = sorted(NATIVE_OPS)
        run_1d_sweep(comm, ops=ops, sizes={"1KB": 256, "1MB": 1 << 19}, warmup=2, iters=5,
                     output_dir=str(tmp_path / "n1d"), impl_name="native", validate=True,
                     batched=True, graph=True, op_opts={"impl": "native"})
        eng = get_native(comm)
        x = make_data((4096,), torch.bfloat16, 0, comm.device)
        ts = eng.time_iters("allreduce", x, x, x.numel(), iters=7, warmup=2)
        assert len(ts) == 7 and all(0 < t < 0.1 for t in ts)
        mean = eng.time_batched("allreduce", x, x, x.numel(), iters=20, warmup=2)
        assert 0 < mean < 0.1
        # stream ordering: an op enqueued from torch's DEFAULT stream (handle 0) must run on it —
        # events around a 256 MiB single-rank copy see the copy (>= 512 MiB of HBM traffic)
        from distributed_llm_backend_benchmark_amd.parallel.collectives import make_op

        big = make_data((1 << 27,), torch.bfloat16, 0, comm.device)
        op = make_op("sendrecv", comm, big, impl="native")
        assert torch.cuda.current_stream().cuda_stream == 0
        op.recv.zero_()
        s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        op.run()
        e0.record()
        e0.synchronize()
        assert s0.elapsed_time(e0) > 0.03, s0.elapsed_time(e0)      # ms
        assert torch.equal(op.recv[-4096:], big[-4096:])
    finally:
        comm.destroy()
    files = sorted(os.listdir(tmp_path / "n1d"))
    errs = [f for f in files if f.endswith(".error.json")]
    assert not errs, [json.load(open(tmp_path / "n1d" / f))["error"] for f in errs]
    assert len(files) == len(ops) * 2
    for f in files:
        d = json.load(open(tmp_path / "n1d" / f))
        assert d["validated"] is True, f
        assert d["op_impl"] == "native"
        assert d["batched_method"] == "hip_graph"


def _car_worker(rank, world, sizes):
    import torch

    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import (ONESHOT, TWOSHOT,
                                                                                CustomAllReduce)

    comm = init_distributed("gloo", device="cuda")
    car = CustomAllReduce(comm, capacity_bytes=8 << 20)
    ok = []
    for n in sizes:
        for algo in (ONESHOT, TWOSHOT):
            for it in range(3):   # several epochs: exercises the double-buffer parity
                xs = [torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(
                    100 * r + it), device="cuda").to(torch.bfloat16) for r in range(world)]
                ref = sum(x.float() for x in xs)
                out = car.all_reduce(xs[rank].clone(), algo=algo)
                torch.cuda.synchronize()
                good = torch.allclose(out.float(), ref, rtol=2e-2, atol=5e-2 * world)
                ok.append((n, algo, it, bool(good), car.check_error()))
            comm.barrier()
    car.close()
    comm.destroy()
    return ok


@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_ranks_on_one_gpu(world):
    """The IPC protocol (flags, epochs, both buffer halves) with 2/4/8 ranks sharing one GPU —
    the compile-time W = 2/4/8 kernels the driver's 8-GPU node runs."""
    res = run_multiprocess(_car_worker, world, args=([2048, 65536, 1 << 20],), timeout=600)
    for r in res:
        for n, algo, it, good, err in r:
            assert good and err == 0, (n, algo, it, good, err)


def _car_reg_worker(rank, world, n):
    import torch

    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import (ONESHOT, TWOSHOT,
                                                                                CustomAllReduce)

    comm = init_distributed("gloo", device="cuda")
    car = CustomAllReduce(comm, capacity_bytes=8 << 20)
    car.self_test()
    ok = [("self_test", car.healthy, car.reg_healthy and car.push_healthy)]
    buf = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    rid = car.register(buf)
    assert car.register(buf) == rid            # idempotent
    # interleave registered calls (grid sizes 1..256) with staging-buffer calls of other grid
    # sizes: the epoch (and buffer half) must stay consistent across workgroups and calls
    plan = [("reg", 256), ("copy2", 7), ("reg", 64), ("copy1", 3), ("reg", 1), ("copy2", 128),
            ("reg", 200), ("push", 256), ("push", 5), ("reg", 256), ("push", 128), ("copy1", 32),
            ("push", 1), ("reg", 33), ("push", 64)]
    for it, (kind, nb) in enumerate(plan):
        xs = [torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(
            1000 * r + it), device="cuda").to(torch.bfloat16) for r in range(world)]
        ref = sum(x.float() for x in xs)
        if kind in ("reg", "push"):
            buf.copy_(xs[rank])
            out = car.all_reduce_registered(buf, rid, nblocks=nb, push=kind == "push")
        else:
            out = car.all_reduce(xs[rank].clone(), algo=ONESHOT if kind == "copy1" else TWOSHOT,
                                 nblocks=nb)
        torch.cuda.synchronize()
        good = torch.allclose(out.float(), ref, rtol=2e-2, atol=5e-2 * world)
        ok.append((kind, nb, bool(good), car.check_error()))
    comm.barrier()
    car.close()
    comm.destroy()
    return ok


@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_registered_ranks_on_one_gpu(world):
    """Registered in-place two-shot, pull form (IPC-mapped user buffers, 3 flag phases) and
    push form (remote writes into peer staging halves), with 2/4/8 ranks sharing one GPU,
    interleaved with staging-buffer calls of different grid sizes."""
    res = run_multiprocess(_car_reg_worker, world, args=(world * 8 * 4096 + world * 8 * 3,),
                           timeout=600)
    for r in res:
        assert r[0] == ("self_test", True, True), r[0]
        for kind, nb, good, err in r[1:]:
            assert good and err == 0, (kind, nb, good, err)


def _car_calibrate_worker(rank, world):
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import CustomAllReduce

    comm = init_distributed("gloo", device="cuda")
    car = CustomAllReduce(comm, capacity_bytes=8 << 20)
    car.self_test()
    cal = car.calibrate(sizes=(4 << 10, 64 << 10, 1 << 20), iters=5)
    live = car.reg_counts()
    res = (cal, car.oneshot_max, car.auto_max, car.reg_max, live)
    comm.barrier()
    car.close()
    comm.destroy()
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_custom_allreduce_calibration_agreed_ranks_on_one_gpu(world):
    """the IPC-vs-RCCL crossovers are measured on the node (rank-max,
    agreed): every rank ends with the identical table and the identical oneshot/auto/reg
    thresholds, every candidate passed its check, and the per-size registrations are released."""
    res = run_multiprocess(_car_calibrate_worker, world, timeout=600)
    cal0 = res[0][0]
    for cal, osm, am, rm, live in res:
        assert cal == cal0
        assert (osm, am, rm) == (cal0["oneshot_max"], cal0["auto_max"], cal0["reg_max"])
        assert live == (0, 0), live
    assert [r["bytes"] for r in cal0["table"]] == [4 << 10, 64 << 10, 1 << 20]
    for row in cal0["table"]:
        assert set(row["us"]) == {"rccl", "oneshot", "twoshot", "reg_pull", "reg_push"}, row
        assert all(v is not None and v > 0 for v in row["us"].values()), row


def _car_lifecycle_worker(rank, world):
    import torch

    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import CustomAllReduce

    comm = init_distributed("gloo", device="cuda")
    car = CustomAllReduce(comm, capacity_bytes=1 << 20)
    torch.cuda.synchronize()
    base_mem = torch.cuda.memory_allocated()
    res = {"base": car.reg_counts()}
    ok = True
    held = []
    for i in range(50):
        n = world * 8 * (1024 + 4096 * (i % 7))          # spread over caching-allocator blocks
        buf = torch.full((n,), float(rank + 1), device="cuda", dtype=torch.bfloat16)
        rid = car.register(buf)
        car.all_reduce_registered(buf, rid, nblocks=8)
        torch.cuda.synchronize()
        ok = ok and bool((buf.float() == world * (world + 1) / 2).all()) and car.check_error() == 0
        if i % 5 == 0:
            held.append((buf, rid))      # some stay live for a while
        else:
            car.deregister(rid)
        del buf
    res["peak"] = car.reg_counts()
    for rid in [r for _, r in held]:
        car.deregister(rid)
    held.clear()                         # (no loop variable may keep the last tensor alive)
    torch.cuda.synchronize()
    res["end"] = car.reg_counts()
    res["mem_delta"] = torch.cuda.memory_allocated() - base_mem
    res["ok"] = ok
    comm.barrier()
    car.close()
    comm.destroy()
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_custom_allreduce_registration_lifecycle(world):
    """50 register / all-reduce / deregister cycles (some registrations held across cycles):
    every peer IPC mapping is closed and every registered tensor released at the end
    (VERDICT r1 item 7)."""
    res = run_multiprocess(_car_lifecycle_worker, world, timeout=600)
    for r in res:
        assert r["ok"]
        assert r["base"] == (0, 0)
        assert r["peak"][0] == 10                     # the held ones
        assert r["end"] == (0, 0), r
        assert r["mem_delta"] == 0, r


def _direct_worker(rank, world, n):
    import torch

    from distributed_llm_backend_benchmark_amd.parallel.collectives import make_data, make_op
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo", device="cuda")
    res = []
    # the full CU-budget matrix at every world (round 5: the 8-rank "stall" was the automatic
    # calibration timing its gloo reference leg, not the IPC kernels; tools/diag/ipc8_probe.py)
    nbs = (None, 3, 256)
    for dt in (torch.bfloat16, torch.float32):
        ins = [make_data((n,), dt, r, torch.device("cuda")) for r in range(world)]
        for name in ("allgather", "reduce_scatter", "alltoall"):
            for nb in nbs:
                op = make_op(name, comm, ins[rank], direct=True, nblocks=nb)
                for _ in range(3):            # repeated calls on one registration
                    op.reset()
                    op.run()
                torch.cuda.synchronize()
                res.append((name, str(dt), nb, op.impl, op.check(ins)))
    # uneven MoE all-to-all (one-hop pulls of this rank's tokens from every peer), tokens x hidden
    for hidden in (1024, 8):
        ins = [make_data((2000, hidden), torch.bfloat16, r, torch.device("cuda"))
               for r in range(world)]
        for nb in (None, 5, 256):
            op = make_op("alltoall_moe", comm, ins[rank], direct=True, nblocks=nb)
            for _ in range(3):
                op.run()
            torch.cuda.synchronize()
            exact = torch.equal(op.result().float(), op.expected(ins))
            res.append(("alltoall_moe", f"h{hidden}", nb, op.impl, exact))
            op.close()
    comm.barrier()
    comm.destroy()
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_direct_ipc_collectives_ranks_on_one_gpu(world):
    """One-hop IPC all-gather / reduce-scatter / all-to-all (registered inputs, entry + exit
    flag barriers) and the uneven MoE all-to-all-v against closed forms (the all-to-alls bit
    exact), 2/4/8 ranks sharing one GPU, bf16 and fp32."""
    res = run_multiprocess(_direct_worker, world, args=(world * 8 * 1000,), timeout=600)
    for r in res:
        for name, dt, nb, impl, ok in r:
            assert impl == "custom" and ok, (name, dt, nb, impl, ok)


def _ddp_custom_worker(rank, world):
    import torch

    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    comm = init_distributed("gloo", device="cuda")
    cfg = GPT2Config(vocab_size=512, block_size=64, n_layer=2, n_head=4, n_embd=256)
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 512, (world * 2, 65), generator=g).cuda()
    local = data[rank * 2:(rank + 1) * 2]
    grads, info = {}, {}
    for ar in ("rccl", "custom"):          # "rccl" = the process group's all_reduce (gloo here)
        m = GPT2(cfg, device=torch.device("cuda"), seed=3)
        tr = FlatParamTrainer(m, comm, lr=1e-3, bucket_mb=0.5, allreduce=ar)
        tr.zero_grad()
        tr._reset()
        m(local[:, :-1], local[:, 1:]).backward()
        tr.finish()
        torch.cuda.synchronize()
        grads[ar] = tr.flat_grad.float().clone()
        for _ in range(3):
            tr.step(local[:, :-1], local[:, 1:])
        torch.cuda.synchronize()
        info[ar] = (len(tr._bucket_reg), len(tr.buckets),
                    comm.all_gather_object(float(tr.master.double().sum())))
        tr.close()
    # hipBLASLt may pick split-K kernels whose reduction order varies run to run: compare the
    # reduced gradients to bf16 resolution, not bit-exactly
    scale = float(grads["rccl"].abs().max())
    err = float((grads["custom"] - grads["rccl"]).abs().max()) / scale
    comm.destroy()
    return err, info["custom"]


def test_ddp_custom_registered_buckets_ranks_on_one_gpu():
    """DDP with allreduce="custom": every bucket IPC-registered and all-reduced in place by the
    two-shot kernel on the comm stream; 2 ranks sharing one GPU. The reduced gradients match the
    process group's all-reduce and the trained weights stay identical across ranks."""
    res = run_multiprocess(_ddp_custom_worker, 2, timeout=600)
    for err, (nreg, nb, sums) in res:
        assert nreg == nb and nb > 1, (nreg, nb)
        assert err < 1e-2, err
        assert len(set(sums)) == 1, sums


@pytest.mark.parametrize("allreduce,fp32_buckets", [("rccl", False), ("custom", False),
                                                    ("auto", False), ("rccl", True)])
def test_ddp_matches_global_batch_and_ranks_stay_identical_ranks_on_one_gpu(allreduce,
                                                                             fp32_buckets):
    """VERDICT r02 weak #7 / item 5, rehearsed with 2 ranks sharing one GPU over a gloo process
    group ("rccl" = the process group's all_reduce): the reduced gradient equals a world-1 run
    on the concatenated global batch, and after three optimizer steps the parameters are
    bitwise identical on every rank. Same worker as the multi-GPU integration test."""
    from ddp_check import ddp_equivalence_worker

    res = run_multiprocess(ddp_equivalence_worker, 2, args=("gloo", allreduce, fp32_buckets),
                           timeout=600)
    tol = 1.5e-2 if fp32_buckets else 3e-2
    for worst, digests, nb in res:
        assert worst < tol, worst
        assert len(set(digests)) == 1, digests
        assert nb > 1


def _tp_rehearsal_worker(rank, world, allreduce, overlap=1, attention="slice", heads=4):
    os.environ["DLBB_GEMM"] = "mfma"                 # the hand-written GEMM on every shape
    os.environ["DLBB_CUSTOM_AR_CALIBRATE"] = "0"     # (calibration has its own test)
    import torch

    from distributed_llm_backend_benchmark_amd import ops as O
    from distributed_llm_backend_benchmark_amd.models.tp_transformer import LLM
    from distributed_llm_backend_benchmark_amd.ops import gemm
    from distributed_llm_backend_benchmark_amd.parallel.comm import Comm, init_distributed

    comm = init_distributed("gloo", device="cuda")
    dev = comm.device
    kw = dict(hidden_size=256, num_layers=2, num_heads=heads, ffn_intermediate=1024, seed=11,
              init_std=0.05)
    # the dense reference runs torch SDPA when the TP model runs our flash kernel
    dense = LLM(comm=Comm(0, 1, 0, "gloo", dev),
                **dict(kw, attention="sdpa" if attention == "flash" else attention))
    reg = allreduce == "custom_reg"
    tp = LLM(comm=comm, allreduce="custom" if reg else allreduce, overlap_chunks=overlap,
             attention=attention, **kw)
    flash_calls = [0]
    real = O.causal_attention

    def counted(qkv, n_head):
        from distributed_llm_backend_benchmark_amd.ops.attention import hip_supported, use_hip
        flash_calls[0] += int(use_hip(qkv) and hip_supported(qkv, n_head))
        return real(qkv, n_head)
    O.causal_attention = counted
    tp.load_from_dense(dense.state_dict())
    if reg:   # every message in the two-shot regime: GEMM into the registered buffer, in place
        tp.ipc_allreduce().oneshot_max = 0
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(2, 64, 256, generator=g, device=dev).to(torch.bfloat16)
    y_ref = dense(x).float()
    y = tp(x).float()
    y2 = tp(x).float()                      # second call: IPC epoch / buffer half flips
    torch.cuda.synchronize()
    car = tp.ipc_allreduce()
    used_custom = car is not None and car.healthy
    errflag = car.check_error() if car is not None else 0
    scale = float(y_ref.abs().max())
    err = max(float((y - y_ref).abs().max()), float((y2 - y_ref).abs().max())) / scale
    mix = gemm.kernel_mix()
    owned = len(car._owned) if car is not None else 0
    O.causal_attention = real
    comm.destroy()
    if attention == "flash":
        return err, flash_calls[0]
    return err, used_custom, errflag, mix["forced"], comm.world_size, owned


@pytest.mark.parametrize("heads", [4, 2])
def test_tp_flash_attention_ranks_on_one_gpu_matches_dense(heads):
    """the TP model's attention="flash" runs our causal flash kernel on each
    rank's fused QKV shard (head dim 64 at 4 heads, 128 at 2 heads; P = 2, one head per rank at
    2 heads) and the all-reduced output equals the dense model on torch SDPA."""
    res = run_multiprocess(_tp_rehearsal_worker, 2, args=("rccl", 1, "flash", heads),
                           timeout=600)
    for err, calls in res:
        assert err < 3e-2, err
        assert calls == 2 * 2, calls          # 2 layers x 2 forwards, every one on the kernel


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("allreduce", ["rccl", "custom", "custom_reg"])
def test_tp_forward_ranks_on_one_gpu_matches_dense(world, allreduce):
    """the TP transformer (reference models.py) with the HIP kernels at
    P = 2 / 4 — column/row-parallel GEMMs on the hand-written MFMA kernel, row-parallel partial
    sums through the process group (gloo over GPU tensors) or the IPC kernel — equals the dense
    world-1 model loaded with the same weights."""
    res = run_multiprocess(_tp_rehearsal_worker, world, args=(allreduce,), timeout=600)
    for err, used_custom, errflag, forced, w, owned in res:
        assert w == world
        assert err < 3e-2, err
        assert forced == "mfma"
        assert errflag == 0
        assert used_custom == (allreduce != "rccl")
        # registered in-place path: one owned buffer (shared by every row-parallel layer)
        assert owned == (1 if allreduce == "custom_reg" else 0), owned


def _run_tp_flash_worker(rank, world, cfg_path):
    from distributed_llm_backend_benchmark_amd.cli import run_tp

    return run_tp.main(["--config", cfg_path, "--backend", "gloo", "--device", "cuda",
                        "--attention", "flash", "--check-dense"])


def test_run_tp_check_dense_flash_ranks_on_one_gpu(tmp_path):
    """``run_tp --attention flash --check-dense`` at P = 2 with both ranks on
    one GPU (gloo over GPU tensors): the flash TP forward equals the dense flash model of the same
    seed, and the run writes the reference's result schema."""
    import json

    import yaml

    cfg = yaml.safe_load(open(os.path.join(REPO, "config", "baseline_config.yaml")))
    cfg["model"].update(hidden_size=512, num_layers=2, num_heads=8, ffn_intermediate=2048,
                        init_std=0.02)
    cfg["input"].update(batch_size=2, sequence_length=256)
    cfg["execution"].update(warmup_iterations=1, benchmark_iterations=3)
    cfg["parallelism"]["world_size"] = 2
    cfg["experiment"]["output_dir"] = str(tmp_path)
    p = tmp_path / "flash.yaml"
    p.write_text(yaml.safe_dump(cfg))
    assert run_multiprocess(_run_tp_flash_worker, 2, args=(str(p),), timeout=600) == [0, 0]
    rec = json.load(open(tmp_path / f"gloo_{cfg['experiment']['name']}.json"))
    assert rec["config"]["execution"]["attention"] == "flash"
    assert rec["throughput"]["dense_check"]["passed"], rec["throughput"]["dense_check"]


def _row_reuse_worker(rank, world):
    os.environ["DLBB_GEMM"] = "mfma"
    os.environ["DLBB_CUSTOM_AR_CALIBRATE"] = "0"
    import torch
    import torch.distributed as dist

    from distributed_llm_backend_benchmark_amd import ops
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.tensor_parallel import RowParallelLinear

    comm = init_distributed("gloo", device="cuda")
    dev = comm.device
    layer = RowParallelLinear(512, 256, comm, generator=torch.Generator(device=dev).manual_seed(
        7 + rank), std=0.05, allreduce="custom")
    car = layer._car
    car.oneshot_max = 0                     # every output through the registered buffer
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    x1, x2 = (torch.randn(2, 64, 256, generator=g, device=dev).to(torch.bfloat16)
              for _ in range(2))
    y1 = layer(x1)
    y2 = layer(x2)                          # a second call must not overwrite y1
    a, _ = layer.launch(x1)                 # the internal path does use the shared buffer
    shared = layer._aliases_registered(a)
    torch.cuda.synchronize()
    errs = []
    for x, y in ((x1, y1), (x2, y2)):
        ref = ops.linear(x, layer.weight).float()
        dist.all_reduce(ref)
        errs.append(float((y.float() - ref).abs().max()) / float(ref.abs().max()))
    owned = len(car._owned)
    distinct = y1.data_ptr() != y2.data_ptr()
    comm.destroy()
    return max(errs), shared, owned, distinct


def test_row_parallel_forward_returns_owned_tensor_ranks_on_one_gpu():
    """RowParallelLinear.forward on the registered IPC path returns an owned tensor
    — y1 = layer(x1); y2 = layer(x2) leaves y1 intact — while launch() stays zero-copy."""
    for err, shared, owned, distinct in run_multiprocess(_row_reuse_worker, 2, timeout=600):
        assert err < 3e-2, err
        assert shared and owned == 1 and distinct


@pytest.mark.parametrize("allreduce", ["rccl", "custom", "custom_reg"])
def test_tp_overlapped_forward_ranks_on_one_gpu_matches_dense(allreduce):
    """The micro-batch interleaved TP forward (overlap_chunks=2: each all-reduce on a side comm
    stream under the other micro-batch's GEMMs) at P = 2 equals the dense model; the registered
    path keeps one IPC buffer per micro-batch in flight."""
    res = run_multiprocess(_tp_rehearsal_worker, 2, args=(allreduce, 2), timeout=600)
    for err, used_custom, errflag, forced, w, owned in res:
        assert err < 3e-2, err
        assert errflag == 0
        assert used_custom == (allreduce != "rccl")
        assert owned == (2 if allreduce == "custom_reg" else 0), owned


def test_run_tp_shard_as_world1(tmp_path):
    """run_tp --shard-as 8 runs rank 0's shard of an 8-way TP model on
    one GPU (per-rank shapes, emulated all-reduce with a link-time stand-in) and writes
    <backend>_<name>_shard8.json."""
    import yaml

    cfg = yaml.safe_load(open(os.path.join(REPO, "config", "1b_config.yaml")))
    cfg["model"]["num_layers"] = 2
    cfg["experiment"]["output_dir"] = str(tmp_path)
    cfg["execution"]["warmup_iterations"] = 2
    cfg["execution"]["benchmark_iterations"] = 3
    cfg["parallelism"]["world_size"] = 8
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(cfg))
    out = subprocess.run([sys.executable, "-m", "distributed_llm_backend_benchmark_amd.cli.run_tp",
                          "--config", str(p), "--backend", "rccl", "--shard-as", "8",
                          "--emulate-busbw", "100"], capture_output=True, text=True,
                         timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.load(open(tmp_path / f"rccl_{cfg['experiment']['name']}_shard8.json"))
    th = rec["throughput"]
    assert th["shard_as"]["P"] == 8 and th["shard_as"]["emulate_busbw_GBps"] == 100
    B, S, H = cfg["input"]["batch_size"], cfg["input"]["sequence_length"], cfg["model"]["hidden_size"]
    assert th["allreduce_bytes_per_forward_per_rank"] == 2 * 2 * B * S * H * 2
    assert th["tokens_per_s"] > 0


@pytest.mark.parametrize("graph", [False, True])
def test_run_tp_shard_as_overlapped(tmp_path, graph):
    """run_tp --shard-as 4 --overlap-chunks 2 (micro-batch interleaved forward: all-reduce
    stand-ins on a side comm stream), eagerly and captured in a HIP graph (fork / join of the
    comm stream inside the capture); the output file carries the _ov2 suffix and the setting."""
    import yaml

    cfg = yaml.safe_load(open(os.path.join(REPO, "config", "1b_config.yaml")))
    cfg["model"]["num_layers"] = 2
    cfg["experiment"]["output_dir"] = str(tmp_path)
    cfg["execution"]["warmup_iterations"] = 2
    cfg["execution"]["benchmark_iterations"] = 3
    cfg["parallelism"]["world_size"] = 4
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(cfg))
    cmd = [sys.executable, "-m", "distributed_llm_backend_benchmark_amd.cli.run_tp",
           "--config", str(p), "--backend", "rccl", "--shard-as", "4", "--overlap-chunks", "2",
           "--emulate-busbw", "100"] + (["--graph"] if graph else ["--eager"])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.load(open(tmp_path / f"rccl_{cfg['experiment']['name']}_shard4_ov2.json"))
    th = rec["throughput"]
    assert th["overlap_chunks"] == 2 and th["hip_graph"] == graph
    B, S, H = cfg["input"]["batch_size"], cfg["input"]["sequence_length"], cfg["model"]["hidden_size"]
    assert th["allreduce_bytes_per_forward_per_rank"] == 2 * 2 * B * S * H * 2
    # the overlapped GEMMs were tuned beside comm: hand-written kernels only
    keys = [t["key"] for t in th["gemm_kernel_mix"]["linear"]["tuned"]]
    assert keys and all(k[-1] == "concurrent" for k in keys), keys
    assert th["gemm_kernel_mix"]["hand_written_time_fraction"] == 1.0


def test_ddp_comm_stream_is_normal_priority():
    """The comm stream is always normal priority: a high-priority one stretched every kernel
    dispatch of the step (the high-priority dispatch trap, profiles/r03_overlap/SUMMARY.md), so
    round 6 removed the option altogether."""
    import warnings

    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel import ddp

    cfg = GPT2Config(vocab_size=256, block_size=32, n_layer=1, n_head=2, n_embd=64)
    m = GPT2(cfg, device=torch.device("cuda"), seed=1)
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        tr = ddp.FlatParamTrainer(m, None, emulate_comm=True)
    assert tr._comm_stream.priority == 0
    tr.close()


def test_bench_py_world1():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "5",
                          "--warmup", "2"], capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 1 and rec["steps"] == 5 and rec["unit"] == "GB/s"
    assert rec["ms_per_step"] > 0
    sweep = rec["allreduce_sweep"]
    assert [e["bytes"] for e in sweep] == [1 << 10, 8 << 10, 64 << 10, 512 << 10, 4 << 20,
                                           32 << 20, 256 << 20, 1 << 30]
    assert all(e["us"] > 0 and e["impl"] in e["us_by_impl"] for e in sweep), sweep
    # one rank: the timed step is real GPU work (out-of-place copy), never an empty in-place call
    # (algBW above the HBM peak), and the IPC kernels' emulation rides along
    assert rec["config"]["impl"] == "native_oop"
    assert 0 < rec["algbw_GBps"] <= 8000.0, rec["algbw_GBps"]
    assert all(e["impl"] == "native_oop" and e["algbw_GBps"] <= 8000.0 for e in sweep), sweep
    emu = rec["virtual_rank_emulation"]
    for w in ("W2", "W8"):
        assert all(v["valid"] and v["us"] > 0 for v in emu[w].values()), emu
    # BASELINE configs 3-5 at P=1 (full default shapes): every cell validated or refused as
    # below the roofline, and the GPT-2-small DDP step measured
    cfgs = rec["baseline_configs"]
    c3 = cfgs["config3_3d_allgather_reduce_scatter"]
    assert "error" not in c3 and len(c3["rows"]) == 4, c3
    for row in c3["rows"]:
        for op in ("allgather", "reduce_scatter"):
            assert row[op]["best"] is not None, row
            assert all("ms" in v or "invalid" in v for v in row[op]["by_impl"].values()), row
    c4 = cfgs["config4_moe_alltoall"]
    assert "error" not in c4 and all(r["best"] for r in c4["rows"]), c4
    c5 = cfgs["config5_gpt2_ddp"]
    assert "error" not in c5 and c5["batch_per_gpu"] == 16 and c5["seq_len"] == 1024, c5
    assert c5["tokens_per_s"] > 0 and c5["ms_per_step"] > 0
    r = c5["by_allreduce"][c5["best"]]
    assert r["loss"] < r["loss_first_step"] + 1.0 and r["bucket_paths"] == {"none": r["buckets"]}


def test_bench_py_two_ranks_rehearsal():
    """bench.py's multi-rank path (candidate agreement, IPC kernel, native-engine refusal of a
    shared GPU) with 2 ranks on one GPU over a gloo process group (DLBB_BENCH_BACKEND=gloo)."""
    from launch_utils import run_torchrun

    env = dict(os.environ, DLBB_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = run_torchrun(2, [os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "5",
                           "--warmup", "2", "--sweep-max-mib", "32", "--grid",
                           "2,1024,1024;1,2048,2048", "--moe", "2048,1024", "--ddp-model",
                           "2,4,256,4096,4,256", "--ddp-steps", "4"], 600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["vs_baseline"] is not None
    assert rec["config"]["impl"].split("/")[0] in ("custom", "custom_reg", "rccl")
    assert rec["p50_latency_us_512B"] > 0
    coll = rec["collectives_same_message"]
    for name in ("allgather", "reduce_scatter", "alltoall"):
        assert set(coll[name]) == {"rccl", "direct_ipc"}, coll
        assert all(v["busbw_GBps"] > 0 for v in coll[name].values()), coll
    sweep = rec["allreduce_sweep"]
    assert [e["bytes"] for e in sweep][-1] == 32 << 20
    # the IPC kernel (staged and registered) is a candidate at every size on 2 ranks
    assert all({"custom", "custom_reg"} <= set(e["us_by_impl"]) for e in sweep), sweep
    assert all(e["busbw_GBps"] > 0 for e in sweep), sweep
    # BASELINE configs 3-5: all three sections present and valid
    cfgs = rec["baseline_configs"]
    c3 = cfgs["config3_3d_allgather_reduce_scatter"]
    assert "error" not in c3 and len(c3["rows"]) == 2, c3
    for row in c3["rows"]:
        for op in ("allgather", "reduce_scatter"):
            cells = row[op]["by_impl"]
            assert "ms" in cells["rccl"] and "ms" in cells["direct_ipc"], cells
            assert row[op]["busbw_GBps"] > 0
    c4 = cfgs["config4_moe_alltoall"]
    assert "error" not in c4 and c4["rows"][0]["busbw_GBps"] > 0, c4
    assert "ms" in c4["rows"][0]["by_impl"]["direct_ipc"], c4     # our all-to-all-v kernel
    c5 = cfgs["config5_gpt2_ddp"]
    assert "error" not in c5 and c5["best"] in ("auto", "rccl", "custom"), c5
    # native RCCL refuses two ranks on one GPU: recorded as an error for that path only
    assert "error" in c5["by_allreduce"]["native"]
    auto = c5["by_allreduce"]["auto"]
    assert "ms_per_step" in auto and sum(auto["bucket_paths"].values()) == auto["buckets"]


def test_tp_forward_world1_matches_torch():
    from distributed_llm_backend_benchmark_amd.models.tp_transformer import LLM
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("rccl")
    try:
        kw = dict(hidden_size=512, num_layers=2, num_heads=8, ffn_intermediate=2048, comm=comm,
                  seed=3, init_std=0.02)
        hip = LLM(kernels="hip", **kw)
        ref = LLM(kernels="torch", **kw)
        x = torch.randn(2, 128, 512, device="cuda", dtype=torch.bfloat16)
        y1, y2 = hip(x), ref(x)
        torch.testing.assert_close(y1.float(), y2.float(), rtol=5e-2, atol=5e-2)
        for ad in ("fp32",):
            hip32 = LLM(kernels="hip", allreduce_dtype=ad, **kw)
            torch.testing.assert_close(hip32(x).float(), y2.float(), rtol=5e-2, atol=5e-2)
    finally:
        comm.destroy()


def test_gpt2_ddp_step_world1():
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    cfg = GPT2Config(vocab_size=1024, block_size=256, n_layer=2, n_head=4, n_embd=256)
    m = GPT2(cfg, device=torch.device("cuda"))
    tr = FlatParamTrainer(m, None, lr=1e-3, bucket_mb=1)
    idx = torch.randint(0, cfg.vocab_size, (4, 256), device="cuda")
    losses = [tr.step(idx, idx) for _ in range(8)]
    assert losses[-1] < losses[0] - 0.5, losses


def test_gpt2_grad_sinks_match_autograd():
    """Gradient sinks: block linears, LayerNorms, the position embedding and the tied token
    embedding / LM head (two uses per step) accumulate in-kernel into the trainer's flat buckets
    (no AccumulateGrad); the flat gradients must
    equal a plain autograd backward of the same model, and every bucket must be counted
    complete exactly once during backward."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    cfg = GPT2Config(vocab_size=1024, block_size=256, n_layer=2, n_head=4, n_embd=256)
    dev = torch.device("cuda")
    idx = torch.randint(0, cfg.vocab_size, (4, 256), device=dev)
    ref = GPT2(cfg, device=dev, seed=11)
    ref(idx, idx).backward()
    m = GPT2(cfg, device=dev, seed=11)
    tr = FlatParamTrainer(m, None, lr=1e-3, bucket_mb=0.25)
    assert sum(hasattr(p, "_dlbb_grad_sink") for p in m.parameters()) == 12 * cfg.n_layer + 4
    for _ in range(2):                      # second pass: buffers reused, zeroed, re-counted
        tr.zero_grad()
        tr._reset()
        m(idx, idx).backward()
        assert all(b.ready == len(b.params) for b in tr.buckets), [
            (b.ready, len(b.params)) for b in tr.buckets]
        tr.finish()
        torch.cuda.synchronize()
        for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            o = tr._offsets[id(p)]
            g = tr.flat_grad[o:o + p.numel()].float().view_as(p)
            err = (g - q.grad.float()).abs().max().item()
            assert err <= 2e-2 * max(1.0, q.grad.float().abs().max().item()), (n, err)
    tr.close()
    assert not any(hasattr(p, "_dlbb_grad_sink") for p in m.parameters())


def test_gpt2_tied_sink_unfused_lm_head_matches_autograd():
    """LM head through linear_train (targets=None: loss computed outside the model): the tied
    weight's LM-head gradient runs on the weight-gradient side stream, the embedding backward
    accumulates into the same buffer on the main stream after waiting for that enqueue — the flat
    gradient of wte must equal plain autograd (repeated: a missing wait shows as a race)."""
    import torch.nn.functional as F

    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    cfg = GPT2Config(vocab_size=4096, block_size=256, n_layer=2, n_head=4, n_embd=256)
    dev = torch.device("cuda")
    idx = torch.randint(0, cfg.vocab_size, (8, 256), device=dev)
    ref = GPT2(cfg, device=dev, seed=12)
    F.cross_entropy(ref(idx).float().view(-1, cfg.vocab_size), idx.view(-1)).backward()
    m = GPT2(cfg, device=dev, seed=12)
    tr = FlatParamTrainer(m, None, lr=1e-3, bucket_mb=0.25)
    assert getattr(m.wte, "_dlbb_grad_stream", None) is not None
    o = tr._offsets[id(m.wte)]
    want = ref.wte.grad.float()
    for _ in range(3):
        tr.zero_grad()
        tr._reset()
        F.cross_entropy(m(idx).float().view(-1, cfg.vocab_size), idx.view(-1)).backward()
        tr.finish()
        torch.cuda.synchronize()
        g = tr.flat_grad[o:o + m.wte.numel()].float().view_as(m.wte)
        err = float((g - want).abs().max())
        assert err <= 2e-2 * max(1.0, float(want.abs().max())), err
    tr.close()


def test_zero2_and_checkpoint_world1_gpu(tmp_path):
    """ZeRO-2 trainer on the GPU (world 1 over RCCL) tracks DDP, and its checkpoint resumes
    bit-exactly with HIP kernels (AdamW, LN, attention, GEMMs) in the loop."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer
    from distributed_llm_backend_benchmark_amd.parallel.zero import ShardedTrainer

    comm = init_distributed("rccl")
    try:
        cfg = GPT2Config(vocab_size=1024, block_size=128, n_layer=2, n_head=4, n_embd=256)
        g = torch.Generator(device="cuda").manual_seed(0)
        data = torch.randint(0, cfg.vocab_size, (6, 4, 129), device="cuda", generator=g)
        ddp = FlatParamTrainer(GPT2(cfg, device=torch.device("cuda"), seed=2), comm, lr=1e-3,
                               bucket_mb=1)
        zero = ShardedTrainer(GPT2(cfg, device=torch.device("cuda"), seed=2), comm, lr=1e-3,
                              bucket_mb=1)
        for s in range(3):
            ld = ddp.step(data[s, :, :-1], data[s, :, 1:])
            lz = zero.step(data[s, :, :-1], data[s, :, 1:])
            assert abs(ld - lz) < 2e-2, (s, ld, lz)
        zero.save_checkpoint(str(tmp_path / "ck"))
        cont = [zero.step(data[s, :, :-1], data[s, :, 1:]) for s in range(3, 6)]
        res = ShardedTrainer(GPT2(cfg, device=torch.device("cuda"), seed=99), comm, lr=1e-3,
                             bucket_mb=1)
        res.load_checkpoint(str(tmp_path / "ck"))
        again = [res.step(data[s, :, :-1], data[s, :, 1:]) for s in range(3, 6)]
        assert cont == again, (cont, again)
        assert torch.equal(zero.master, res.master)
    finally:
        comm.destroy()


def test_gpt2_training_step_hip_graph_matches_eager():
    """Whole training step (fwd + bwd + AdamW with the device step counter) captured in a HIP
    graph and replayed tracks the eager trainer step for step."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    cfg = GPT2Config(vocab_size=1024, block_size=128, n_layer=2, n_head=4, n_embd=256)
    g = torch.Generator(device="cuda").manual_seed(5)
    data = torch.randint(0, cfg.vocab_size, (7, 4, 129), device="cuda", generator=g)
    ea = FlatParamTrainer(GPT2(cfg, device=torch.device("cuda"), seed=4), None, lr=1e-3)
    gr = FlatParamTrainer(GPT2(cfg, device=torch.device("cuda"), seed=4), None, lr=1e-3)
    eager = [ea.step(data[s, :, :-1], data[s, :, 1:]) for s in range(7)]
    gr.step(data[0, :, :-1], data[0, :, 1:])
    replay = gr.capture_step(data[1, :, :-1], data[1, :, 1:])      # runs step 1 eagerly
    graphed = [float(replay(data[s, :, :-1], data[s, :, 1:]).item()) for s in range(2, 7)]
    assert gr.step_count == 7 and gr.opt.t == 7
    for a, b in zip(eager[2:], graphed):
        assert abs(a - b) < 2e-2, (eager[2:], graphed)
    assert float((ea.master - gr.master).abs().max()) < 5e-3


def test_ddp_emulated_comm_is_numerically_transparent():
    """The single-GPU overlap measurement (bucket + zeros -> bucket on the comm stream at each
    bucket-ready hook, CU budget comm_blocks) must not change training: same losses and masters
    bit for bit as the plain world-1 step."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.ops.elementwise import reduce_sum
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    dev = torch.device("cuda", 0)
    x = [torch.randn(1 << 16, device=dev).to(torch.bfloat16) for _ in range(2)]
    assert torch.equal(reduce_sum(x, nblocks=3), reduce_sum(x))
    cfg = GPT2Config(vocab_size=512, block_size=64, n_layer=2, n_head=4, n_embd=256)
    idx = torch.randint(0, cfg.vocab_size, (4, 65), device=dev)
    out = []
    for emulate in (False, True):
        tr = FlatParamTrainer(GPT2(cfg, device=dev, seed=5), None, lr=1e-3, bucket_mb=0.1,
                              emulate_comm=emulate, comm_blocks=8 if emulate else None)
        assert len(tr.buckets) > 1
        losses = [tr.step(idx[:, :-1], idx[:, 1:]) for _ in range(3)]
        torch.cuda.synchronize()
        out.append((losses, tr.master.clone()))
        tr.close()
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1])


def test_collectives_sweep_pipeline_ranks_on_one_gpu(tmp_path):
    """VERDICT r03 item 6 rehearsed: cli.collectives 1D (9 ops, --validate) and 3D (RCCL-path and
    --direct-ipc) with 2 ranks sharing one GPU over a gloo process group, then cli.stats and
    cli.compare against the reference CSVs — the code test_collectives_sweep_across_gpus runs."""
    from sweep_pipeline import check_pipeline, run_pipeline

    res = run_pipeline(tmp_path, 2, backend="gloo", device="cuda", direct_ipc=True, timeout=600)
    check_pipeline(res, 2)


def test_allgather_list_form_unpack_bit_exact_world1():
    """List-form all-gather (reference collectives/1d/dsccl.py:72-76) on RCCL: one
    all_gather_into_tensor into a staging buffer, then the list unpack as ONE chunk-copy launch
    (csrc/flatten.hip) — bit-exact at 16-B aligned and unaligned slice offsets."""
    from distributed_llm_backend_benchmark_amd.parallel.collectives import make_data, make_op
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("rccl")
    try:
        for n in (1, 7, 4096, 1000003, 1 << 24):
            x = make_data((n,), torch.bfloat16, 0, comm.device)
            op = make_op("allgather", comm, x, form="list")
            for o in op.outs:
                o.fill_(float("nan"))
            op.run()
            torch.cuda.synchronize()
            assert op._tensor_ok                 # staged + chunk-copy path, not the list call
            assert len(op.outs) == 1 and torch.equal(op.outs[0], x), n
            assert torch.equal(op.result(), x.reshape(-1))
    finally:
        comm.destroy()


@pytest.mark.parametrize("mode", [1, 2])
def test_ddp_overlapped_optimizer_is_bit_exact(mode):
    """Split optimizer with per-bucket AdamW issued during backward (opt_overlap 1: own stream,
    2: on the weight-gradient side stream) must give the same losses and masters, bit for bit, as
    the head range updated after backward — eager and as a captured HIP graph; the step count
    advances once per step."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    dev = torch.device("cuda", 0)
    cfg = GPT2Config(vocab_size=512, block_size=64, n_layer=3, n_head=4, n_embd=256)
    g = torch.Generator(device="cuda").manual_seed(3)
    data = torch.randint(0, cfg.vocab_size, (6, 4, 65), device=dev, generator=g)
    out = []
    for ov in (0, mode):
        tr = FlatParamTrainer(GPT2(cfg, device=dev, seed=6), None, lr=1e-3, bucket_mb=0.3)
        tr.opt_overlap = ov
        assert len(tr.buckets) > 2 and tr._split_optimizer_ok()
        losses = [tr.step(data[s, :, :-1], data[s, :, 1:]) for s in range(3)]
        if ov:
            assert tr._opt_issued == len(tr.buckets) - 1 and tr._opt_stream is not None
        replay = tr.capture_step(data[3, :, :-1], data[3, :, 1:])
        losses += [float(replay(data[s, :, :-1], data[s, :, 1:]).item()) for s in (4, 5)]
        torch.cuda.synchronize()
        assert tr.opt.t == 6 and int(tr.opt.t_dev.item()) == 6
        out.append((losses, tr.master.clone()))
        tr.close()
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1])


def test_unit_upstream_mark_is_bit_exact():
    """Marking the fused LM-head loss as the backward root skips the upstream-gradient scaling
    passes; gradients and loss must be bit-identical to the unmarked backward."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.ops.xent import mark_unit_upstream

    cfg = GPT2Config(vocab_size=1024, block_size=128, n_layer=2, n_head=4, n_embd=256)
    dev = torch.device("cuda")
    idx = torch.randint(0, cfg.vocab_size, (4, 129), device=dev)
    out = []
    for mark in (False, True):
        m = GPT2(cfg, device=dev, seed=21)
        loss = m(idx[:, :-1], idx[:, 1:])
        assert mark_unit_upstream(loss) if mark else True
        loss.backward()
        torch.cuda.synchronize()
        out.append((loss.detach().clone(), [p.grad.clone() for p in m.parameters()]))
    assert torch.equal(out[0][0], out[1][0])
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.equal(a, b)
    ref = GPT2(cfg, device=dev, seed=21)
    assert not mark_unit_upstream(ref(idx[:, :-1], idx[:, 1:]) * 2.0)   # not the fused output


def test_side_stream_recheck_replaces_a_serialised_stream():
    """The warm-up re-check finds a weight-gradient stream that no longer runs beside the
    compute stream (here: forced onto the compute stream itself), replaces it with a verified
    one everywhere it is referenced, and training continues."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel import streams
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    streams.reset()       #  no side streams of earlier tests hold the free queues
    dev = torch.device("cuda", 0)
    cfg = GPT2Config(vocab_size=512, block_size=64, n_layer=2, n_head=4, n_embd=256)
    tr = FlatParamTrainer(GPT2(cfg, device=dev, seed=2), None, lr=1e-3, bucket_mb=0.3)
    idx = torch.randint(0, cfg.vocab_size, (4, 65), device=dev)
    tr.step(idx[:, :-1], idx[:, 1:])
    cur = torch.cuda.current_stream(dev)
    old = tr._wgrad_stream
    for p in tr._params:
        if getattr(p, "_dlbb_grad_stream", None) is old:
            p._dlbb_grad_stream = cur
    tr._wgrad_streams[0] = cur
    tr._wgrad_stream = cur
    tr._recheck_side_streams()
    rec = tr.side_stream_checks[-1]
    assert rec["serialised"] == 1 and rec["replaced"] == [0], rec
    assert tr._wgrad_stream is not cur
    assert rec["now_concurrent"] is True, rec
    assert all(getattr(p, "_dlbb_grad_stream", None) is not cur for p in tr._params)
    losses = [tr.step(idx[:, :-1], idx[:, 1:]) for _ in range(3)]
    assert losses[-1] < losses[0] + 0.5
    tr.close()
