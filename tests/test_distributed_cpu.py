"""Multi-process CPU tests over Gloo (BASELINE config 1: "gloo backend world_size=2 on CPU").

The reference's smoke tests need mpirun/deepspeed and a real backend (test/test_open.py,
test/test_deepseed.py); here every collective, the sweep engine + JSON schema + timing gather,
tensor parallelism and DDP are checked with world_size 2 (and 4) Gloo processes on localhost.
"""

import json
import os

import pytest
import torch

from mp_utils import run_multiprocess


def _sweep_worker(rank, world, outdir):
    from distributed_llm_backend_benchmark_amd.bench.sweep import run_1d_sweep, run_3d_sweep
    from distributed_llm_backend_benchmark_amd.parallel.collectives import OPS
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo")
    ops = list(OPS)
    run_1d_sweep(comm, ops=ops, sizes={"1KB": 256, "4KiB": 2048}, dtype="fp32", warmup=2,
                 iters=4, output_dir=os.path.join(outdir, "1d"), impl_name="gloo",
                 validate=True, batched=True)
    run_3d_sweep(comm, ops=["allreduce", "allgather", "reduce_scatter", "broadcast", "reduce",
                            "gather", "alltoall"],
                 batch_sizes=[1, 2], seq_lengths=[4], hidden_dims=[64], dtype="bf16",
                 warmup=1, iters=3, output_dir=os.path.join(outdir, "3d"), impl_name="gloo",
                 validate=True)
    # the reference's 3D MPI form: bf16 data on an fp32 wire, validated against the same
    # bf16-rounded values (round 5: the closed form used to regenerate unrounded fp32 data)
    run_3d_sweep(comm, ops=["allreduce", "allgather", "reduce_scatter"], batch_sizes=[1],
                 seq_lengths=[4], hidden_dims=[64], dtype="bf16", wire_dtype="fp32",
                 warmup=1, iters=2, output_dir=os.path.join(outdir, "3d_wire"),
                 impl_name="gloo", validate=True)
    # resume: nothing rewritten
    again = run_1d_sweep(comm, ops=["allreduce"], sizes={"1KB": 256}, dtype="fp32", warmup=1,
                         iters=2, output_dir=os.path.join(outdir, "1d"), impl_name="gloo",
                         resume=True)
    comm.destroy()
    return len(again)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_sweeps_all_ops(tmp_path, world):
    from distributed_llm_backend_benchmark_amd.stats import stats1d, stats3d

    res = run_multiprocess(_sweep_worker, world, args=(str(tmp_path),), timeout=600)
    assert res == [0] * world          # resume skipped the existing config
    d1 = tmp_path / "1d"
    files = sorted(os.listdir(d1))
    errors = {f: json.load(open(d1 / f))["error"] for f in files if f.endswith(".error.json")}
    assert not errors, errors
    from distributed_llm_backend_benchmark_amd.parallel.collectives import OPS
    assert len(files) == len(OPS) * 2
    for f in files:
        rec = json.load(open(d1 / f))
        assert rec["validated"] is True, f
        assert len(rec["timings"]) == world and all(len(t) == 4 for t in rec["timings"])
        assert rec["timing_method"] == "host_perf_counter"
        assert rec["batched_mean_s"] > 0
    wire = sorted(os.listdir(tmp_path / "3d_wire"))
    assert wire and not [f for f in wire if f.endswith(".error.json")], wire
    assert all(json.load(open(tmp_path / "3d_wire" / f))["validated"] is True for f in wire)
    rows = stats1d.process_directory(str(d1), str(tmp_path / "s1d"), verbose=False)
    assert len(rows) == len(files)
    ar = [r for r in rows if r["operation"] == "allreduce" and r["data_size_name"] == "4KiB"][0]
    assert ar["bytes"] == 8192 and ar["busbw_gbps"] > 0
    d3 = tmp_path / "3d"
    f3 = os.listdir(d3)
    assert not [f for f in f3 if f.endswith(".error.json")], f3
    assert len(f3) == 7 * 2
    rows3 = stats3d.process_directory(str(d3), str(tmp_path / "s3d"), "gloo", verbose=False)
    assert all(r["validated"] if "validated" in r else True for r in rows3)


def _tp_worker(rank, world, attention):
    from distributed_llm_backend_benchmark_amd.models.tp_transformer import LLM
    from distributed_llm_backend_benchmark_amd.parallel.comm import Comm, init_distributed

    comm = init_distributed("gloo")
    kw = dict(hidden_size=128, num_layers=2, num_heads=4, ffn_intermediate=512, seed=11,
              init_std=0.05, attention=attention)
    dense = LLM(comm=Comm(0, 1, 0, "gloo", torch.device("cpu")), **kw)
    tp = LLM(comm=comm, **kw)
    tp.load_from_dense(dense.state_dict())
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 128, generator=g).to(torch.bfloat16)
    y_ref = dense(x).float()
    y_tp = tp(x).float()
    err = float((y_ref - y_tp).abs().max())
    tp32 = LLM(comm=comm, allreduce_dtype="fp32", **kw)
    tp32.load_from_dense(dense.state_dict())
    err32 = float((tp32(x).float() - y_ref).abs().max())
    nbytes = tp.comm_bytes()
    # micro-batch interleaved forward: same weights, same result (per-token math is unchanged;
    # the all-reduces just run in a different order)
    tpo = LLM(comm=comm, overlap_chunks=2, **kw)
    tpo.load_from_dense(dense.state_dict())
    y_ov = tpo(x).float()
    ov_diff = float((y_ov - y_tp).abs().max())
    ov_split = tpo.overlap_split(x)
    odd = tpo.overlap_split(x[:1])              # batch 1 does not split: plain forward
    comm.destroy()
    return err, err32, nbytes, ov_diff, ov_split, odd, tpo.comm_bytes()


@pytest.mark.parametrize("attention", ["slice", "sdpa"])
def test_tensor_parallel_matches_dense(attention):
    res = run_multiprocess(_tp_worker, 2, args=(attention,), timeout=300)
    for err, err32, nbytes, ov_diff, ov_split, odd, ov_bytes in res:
        assert err < 0.1 and err32 < 0.1, (err, err32)
        assert nbytes == 2 * 2 * (2 * 16 * 128 * 2)   # 2 layers x 2 AR x [B,S,H] bf16
        assert ov_split == 2 and odd == 1
        assert ov_diff == 0.0, ov_diff
        assert ov_bytes == nbytes


def _ddp_worker(rank, world, bucket_mb, overlap, mode):
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    comm = init_distributed("gloo")
    cfg = GPT2Config(vocab_size=256, block_size=32, n_layer=2, n_head=2, n_embd=64)
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (world * 2, 33), generator=g)
    local = data[rank * 2:(rank + 1) * 2]
    # reference gradient on the FULL batch in one process (mean over ranks == global mean)
    ref = GPT2(cfg, seed=3)
    loss = ref(data[:, :-1], data[:, 1:])
    loss.backward()
    ref_grads = {n: p.grad.float().clone() for n, p in ref.named_parameters()}
    m = GPT2(cfg, seed=3)
    tr = FlatParamTrainer(m, comm, lr=1e-3, bucket_mb=bucket_mb, overlap=overlap, mode=mode)
    tr.zero_grad()
    tr._reset()
    l = m(local[:, :-1], local[:, 1:])
    l.backward()
    tr.finish()
    errs = []
    for n, p in m.named_parameters():
        o = tr._offsets[id(p)]
        gavg = tr.flat_grad[o:o + p.numel()].float().view_as(p) / world
        errs.append(float((gavg - ref_grads[n]).abs().max()))
    nb = len(tr.buckets)
    tr.opt.step(tr.flat_grad, working_bf16=tr.flat_param, grad_scale=1.0 / world)
    for _ in range(2):
        tr.step(local[:, :-1], local[:, 1:])
    # parameters must stay bit-identical across ranks
    chk = comm.all_gather_object(float(tr.master.double().sum()))
    comm.destroy()
    return max(errs), nb, chk


@pytest.mark.parametrize("bucket_mb,overlap,mode", [(0.05, True, "view"), (100, False, "view"),
                                                    (0.05, True, "flatten")])
def test_ddp_grads_match_full_batch(bucket_mb, overlap, mode):
    res = run_multiprocess(_ddp_worker, 2, args=(bucket_mb, overlap, mode), timeout=300)
    for err, nb, chk in res:
        assert err < 2e-2, err
        assert len(set(chk)) == 1
    if bucket_mb < 1:
        assert res[0][1] > 1


def _zero_worker(rank, world):
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer
    from distributed_llm_backend_benchmark_amd.parallel.zero import ShardedTrainer

    comm = init_distributed("gloo")
    cfg = GPT2Config(vocab_size=256, block_size=32, n_layer=2, n_head=2, n_embd=64)
    g = torch.Generator().manual_seed(1)
    data = torch.randint(0, 256, (world * 2, 33), generator=g)
    local = data[rank * 2:(rank + 1) * 2]
    md, mz = GPT2(cfg, seed=9), GPT2(cfg, seed=9)
    ddp = FlatParamTrainer(md, comm, lr=1e-3, bucket_mb=0.05)
    zero = ShardedTrainer(mz, comm, lr=1e-3, bucket_mb=0.05)
    assert zero.shard_numel * world == zero.numel
    for _ in range(3):
        ld = ddp.step(local[:, :-1], local[:, 1:])
        lz = zero.step(local[:, :-1], local[:, 1:])
    # the all-gathered bf16 parameters must match DDP's, parameter by parameter
    diff = max(float((a.float() - b.float()).abs().max())
               for a, b in zip(md.parameters(), mz.parameters()))
    # and the sharded optimizer really holds 1/world of the state
    errs = [zero.master.numel() * world - zero.numel]
    comm.destroy()
    return diff, max(errs), ld, lz


def test_zero2_matches_ddp():
    res = run_multiprocess(_zero_worker, 2, timeout=300)
    for diff, err, ld, lz in res:
        assert diff < 2e-2 and err == 0, (diff, err)
        assert abs(ld - lz) < 1e-2


def _ckpt_worker(rank, world, ckdir, zero):
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer
    from distributed_llm_backend_benchmark_amd.parallel.zero import ShardedTrainer

    comm = init_distributed("gloo")
    cfg = GPT2Config(vocab_size=256, block_size=16, n_layer=2, n_head=2, n_embd=64)
    g = torch.Generator().manual_seed(3)
    data = torch.randint(0, 256, (4, world * 2, 17), generator=g)
    local = data[:, rank * 2:(rank + 1) * 2]
    cls = ShardedTrainer if zero else FlatParamTrainer

    def trainer(seed):
        return cls(GPT2(cfg, seed=seed), comm, lr=1e-3, bucket_mb=0.05)

    a = trainer(5)                        # continuous: 4 steps
    for s in range(4):
        a.step(local[s, :, :-1], local[s, :, 1:])
    b = trainer(5)                        # 2 steps, checkpoint
    for s in range(2):
        b.step(local[s, :, :-1], local[s, :, 1:])
    b.save_checkpoint(ckdir)
    c = trainer(77)                       # different init, resumed from the checkpoint
    c.load_checkpoint(ckdir)
    assert c.step_count == 2 and c.opt.t == 2
    for s in range(2, 4):
        c.step(local[s, :, :-1], local[s, :, 1:])
    diff = max(float((x.float() - y.float()).abs().max())
               for x, y in zip(a.model.parameters(), c.model.parameters()))
    mdiff = float((a.master - c.master).abs().max())
    files = sorted(os.listdir(ckdir))
    comm.destroy()
    return diff, mdiff, files


@pytest.mark.parametrize("zero", [False, True])
def test_checkpoint_resume_bit_exact(tmp_path, zero):
    res = run_multiprocess(_ckpt_worker, 2, args=(str(tmp_path / "ck"), zero), timeout=300)
    for diff, mdiff, files in res:
        assert diff == 0.0 and mdiff == 0.0, (diff, mdiff)
        want = {"meta.json", "rank00000.safetensors"} | ({"rank00001.safetensors"} if zero
                                                          else set())
        assert set(files) == want, files


def _fault_worker(rank, world, outdir, spec):
    os.environ["DLBB_FAULT_INJECT"] = spec
    from distributed_llm_backend_benchmark_amd.bench.sweep import run_1d_sweep
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo")
    written = run_1d_sweep(comm, ops=["allreduce", "broadcast"],
                           sizes={"1KB": 256, "4KiB": 2048}, dtype="fp32", warmup=1, iters=2,
                           output_dir=outdir, impl_name="gloo")
    comm.destroy()
    return [os.path.basename(w) for w in written]


@pytest.mark.parametrize("spec", ["op=allreduce,size=1KB,rank=1,stage=setup",
                                  "op=broadcast,size=4KiB,stage=run"])
def test_fault_injection_records_error_and_continues(tmp_path, spec):
    out = str(tmp_path / "f")
    res = run_multiprocess(_fault_worker, 2, args=(out, spec), timeout=300)
    assert len(res[0]) == 3                       # the other three configs completed
    errs = [f for f in os.listdir(out) if f.endswith(".error.json")]
    assert len(errs) == 1
    rec = json.load(open(os.path.join(out, errs[0])))
    assert "injected fault" in rec["error"]


def _corrupt_worker(rank, world, outdir, spec):
    os.environ["DLBB_FAULT_INJECT"] = spec
    from distributed_llm_backend_benchmark_amd.bench.sweep import run_1d_sweep, run_3d_sweep
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo")
    w1 = run_1d_sweep(comm, ops=["allreduce", "allgather"], sizes={"1KB": 256, "4KiB": 2048},
                      dtype="fp32", warmup=1, iters=2, output_dir=outdir + "/1d",
                      impl_name="gloo", validate=True)
    w3 = run_3d_sweep(comm, ops=["allreduce"], batch_sizes=[1], seq_lengths=[4, 8],
                      hidden_dims=[64], dtype="fp32", warmup=1, iters=2,
                      output_dir=outdir + "/3d", impl_name="gloo", validate=True)
    comm.destroy()
    return [os.path.basename(w) for w in w1 + w3]


def test_wrong_result_never_becomes_a_statistic(tmp_path):
    """a collective whose output fails validation (injected on rank 1 with
    DLBB_FAULT_INJECT stage=corrupt) is written as <stem>.error.json with invalid=wrong_result,
    no result file; and a raw record carrying validated=false is refused by BOTH stats stages."""
    from distributed_llm_backend_benchmark_amd.stats import stats1d, stats3d

    out = str(tmp_path / "c")
    spec = "op=allreduce,rank=1,stage=corrupt"
    written = run_multiprocess(_corrupt_worker, 2, args=(out, spec), timeout=300)[0]
    assert sorted(written) == ["gloo_allgather_ranks2_1KB.json",
                               "gloo_allgather_ranks2_4KiB.json"], written
    for sub, n in (("1d", 2), ("3d", 2)):
        errs = [f for f in os.listdir(f"{out}/{sub}") if f.endswith(".error.json")]
        assert len(errs) == n, errs
        for f in errs:
            rec = json.load(open(f"{out}/{sub}/{f}"))
            assert rec["invalid"] == "wrong_result" and rec["validated"] is False
            assert not os.path.exists(f"{out}/{sub}/{f[:-len('.error.json')]}.json")
    # the stats stages refuse a raw record whose validation failed, even if someone wrote one
    good = json.load(open(f"{out}/1d/gloo_allgather_ranks2_1KB.json"))
    assert good["validated"] is True
    assert stats1d.refused(good) is None
    bad = dict(good, operation="allreduce", validated=False)
    assert stats1d.refused(bad) == "wrong_result"
    os.makedirs(f"{out}/raw1", exist_ok=True)
    json.dump(bad, open(f"{out}/raw1/gloo_allreduce_ranks2_1KB.json", "w"))
    json.dump(good, open(f"{out}/raw1/gloo_allgather_ranks2_1KB.json", "w"))
    rows = stats1d.process_directory(f"{out}/raw1", f"{out}/s1", verbose=False)
    assert [r["operation"] for r in rows] == ["allgather"]
    os.makedirs(f"{out}/raw3", exist_ok=True)
    rec3 = {"implementation": "gloo", "operation": "allreduce", "num_ranks": 2,
            "tensor_shape": {"batch": 1, "seq_len": 4, "hidden_dim": 64}, "num_elements": 256,
            "tensor_size_bytes": 1024, "tensor_size_mb": 0.001, "dtype": "float32",
            "timings": [[1e-3, 1e-3], [1e-3, 1e-3]], "validated": False}
    json.dump(rec3, open(f"{out}/raw3/gloo_allreduce_ranks2_b1_s4_h64.json", "w"))
    json.dump(dict(rec3, validated=True, num_elements=512, tensor_size_bytes=2048,
                   tensor_shape={"batch": 1, "seq_len": 8, "hidden_dim": 64}),
              open(f"{out}/raw3/gloo_allreduce_ranks2_b1_s8_h64.json", "w"))
    rows3 = stats3d.process_directory(f"{out}/raw3", f"{out}/s3", "gloo", verbose=False)
    assert [r["seq_len"] for r in rows3] == [8]


def _experiment_worker(rank, world):
    from distributed_llm_backend_benchmark_amd.data import create_dataset_from_config
    from distributed_llm_backend_benchmark_amd.models.tp_transformer import create_model_from_config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.utils.config import DEFAULT_CONFIG, validate_config
    from distributed_llm_backend_benchmark_amd.utils.metrics import (
        MetricsCollector, gather_metrics_from_all_ranks, run_experiment)
    import copy

    comm = init_distributed("gloo")
    cfg = copy.deepcopy(DEFAULT_CONFIG)
    cfg["model"].update(hidden_size=64, num_layers=1, num_heads=2, ffn_intermediate=128)
    cfg["input"].update(batch_size=1, sequence_length=8)
    cfg["execution"].update(warmup_iterations=1, benchmark_iterations=3)
    cfg["parallelism"]["world_size"] = world
    cfg = validate_config(cfg)
    model = create_model_from_config(cfg, comm)
    ds = create_dataset_from_config(cfg, comm.device)
    m = run_experiment(model, ds, cfg, MetricsCollector(rank, world), comm)
    m.record_init_time(0.0)
    s = m.get_summary()
    g = gather_metrics_from_all_ranks(comm, s)
    comm.destroy()
    return len(m.metrics["forward_times"]), g


def test_run_experiment_and_gather_metrics():
    res = run_multiprocess(_experiment_worker, 2, timeout=300)
    assert res[0][0] == 3 and res[1][1] is None
    g = res[0][1]
    assert len(g["forward_mean_per_rank"]) == 2 and len(g["forward_p95_per_rank"]) == 2
    assert g["coefficient_of_variation"] >= 0


def _mode_worker(rank, world):
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    comm = init_distributed("gloo")
    cfg = GPT2Config(vocab_size=256, block_size=16, n_layer=2, n_head=2, n_embd=64)
    g = torch.Generator().manual_seed(4)
    data = torch.randint(0, 256, (4, world * 2, 17), generator=g)
    local = data[:, rank * 2:(rank + 1) * 2]
    out = {}
    for mode in ("view", "flatten"):
        tr = FlatParamTrainer(GPT2(cfg, seed=6), comm, lr=1e-3, bucket_mb=0.05, mode=mode)
        for s in range(4):
            tr.step(local[s, :, :-1], local[s, :, 1:])
        out[mode] = tr.master.clone()
        tr.close()
    comm.destroy()
    return float((out["view"] - out["flatten"]).abs().max())


def test_flatten_mode_matches_view_mode_over_steps():
    """Regression: flatten mode must pick up each step's freshly allocated .grad tensors."""
    for d in run_multiprocess(_mode_worker, 2, timeout=300):
        assert d < 1e-6, d


def test_bench_py_gloo_world2_contract():
    """bench.py under torchrun on the CPU (gloo, world 2, small message): the driver's JSON
    contract — one line, the BASELINE metric, busBW > 0 at P = 2, vs_baseline set, the
    all-reduce size sweep present."""
    import json
    import subprocess
    import sys

    from launch_utils import run_torchrun

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--shape", "1,64,256", "--sweep-max-mib", "1"]
    env = {k: v for k, v in os.environ.items() if k not in ("CUDA_VISIBLE_DEVICES",)}
    out = run_torchrun(2, cmd, 300, env=env, cwd=repo)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["metric"] == "all-reduce bus BW (GB/s)" and rec["n_gpus"] == 2
    assert rec["value"] > 0 and rec["vs_baseline"] is not None and rec["steps"] == 3
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert [e["bytes"] for e in rec["allreduce_sweep"]] == [1 << 10, 8 << 10, 64 << 10, 512 << 10]
    assert all(e["impl"] == "rccl" and e["busbw_GBps"] > 0 for e in rec["allreduce_sweep"])


def test_bench_py_deadline_keeps_the_headline():
    """with a whole-run deadline that has already passed, bench.py (gloo,
    world 2) still measures and prints the one valid headline line; everything after it is
    recorded as skipped_deadline, and the run's wall time is in the record."""
    import json
    import subprocess
    import sys

    from launch_utils import run_torchrun

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--shape", "1,64,256", "--sweep-max-mib", "1", "--deadline-s", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("CUDA_VISIBLE_DEVICES",)}
    out = run_torchrun(2, cmd, 300, env=env, cwd=repo)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["metric"] == "all-reduce bus BW (GB/s)" and rec["value"] > 0
    assert rec["steps"] == 3 and rec["deadline_s"] == 0 and rec["wall_s"] > 0
    assert rec["side_skipped_deadline"] is True
    assert all(e.get("skipped_deadline") for e in rec["allreduce_sweep"])
    assert all(v == {"skipped_deadline": True} for v in rec["baseline_configs"].values())
    assert "config5_gpt2_ddp" in rec["skipped_deadline"]
    assert any(k.startswith("allreduce_sweep/") for k in rec["skipped_deadline"])


def _precision_worker(rank, world, grad_dtype_name):
    """Reduction error of the DDP gradient all-reduce alone: flatten-mode buckets (bf16 or fp32)
    reduced through the process group vs the exact fp64 mean of every rank's local bf16
    gradient (all-gathered)."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    gd = {"bf16": torch.bfloat16, "fp32": torch.float32}[grad_dtype_name]
    comm = init_distributed("gloo")
    cfg = GPT2Config(vocab_size=256, block_size=32, n_layer=2, n_head=2, n_embd=64)
    g = torch.Generator().manual_seed(21)
    data = torch.randint(0, 256, (world * 2, 33), generator=g)
    local = data[rank * 2:(rank + 1) * 2]
    m = GPT2(cfg, seed=4)
    tr = FlatParamTrainer(m, comm, lr=1e-3, bucket_mb=0.05, mode="flatten", grad_dtype=gd)
    assert tr.flat_grad.dtype == gd
    tr.zero_grad()
    tr._reset()
    m(local[:, :-1], local[:, 1:]).backward()
    tr.finish()
    worst = 0.0
    for p in tr._params:
        mine = p.grad.double().reshape(-1)
        every = [torch.empty_like(mine) for _ in range(world)]
        torch.distributed.all_gather(every, mine)
        exact = torch.stack(every).mean(0)
        o = tr._offsets[id(p)]
        got = tr.flat_grad[o:o + p.numel()].double() / world
        scale = float(exact.abs().max()) or 1.0
        worst = max(worst, float((got - exact).abs().max()) / scale)
    comm.destroy()
    return worst


def test_ddp_reduction_precision_world8():
    """P = 8 (the driver's scaling node): bf16 gradient buckets are summed in bf16 by the
    collective, fp32 buckets (mode='flatten', grad_dtype=fp32) in fp32. Pins the max error of
    the averaged gradient relative to each tensor's largest entry."""
    bf = run_multiprocess(_precision_worker, 8, args=("bf16",), timeout=600)
    fp = run_multiprocess(_precision_worker, 8, args=("fp32",), timeout=600)
    worst_bf, worst_fp = max(bf), max(fp)         # per-rank worst errors
    print(f"P=8 averaged-gradient max rel error: bf16 buckets {worst_bf:.3e}, "
          f"fp32 buckets {worst_fp:.3e}")
    assert worst_fp < 1e-6, worst_fp          # fp32 sum of bf16 values (measured 3.0e-8)
    assert worst_bf < 3e-2, worst_bf          # 8-way bf16 sum: a few bf16 ulps (measured 8.2e-3)
    assert worst_fp < worst_bf


def test_view_mode_rejects_non_param_grad_dtype():
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    m = GPT2(GPT2Config(vocab_size=64, block_size=8, n_layer=1, n_head=1, n_embd=32), seed=1)
    with pytest.raises(ValueError, match="mode='flatten'"):
        FlatParamTrainer(m, None, mode="view", grad_dtype=torch.float32)


def test_rccl_init_refuses_more_ranks_than_gpus(monkeypatch):
    """RCCL needs one GPU per rank: a LOCAL_RANK beyond the visible devices fails at init with
    the reason (instead of a late duplicate-device error from RCCL)."""
    from distributed_llm_backend_benchmark_amd.parallel import comm as C

    monkeypatch.setattr(C.torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(C.torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("MASTER_PORT", "1")
    with pytest.raises(RuntimeError, match="one GPU per rank"):
        C.init_distributed("rccl")


@pytest.mark.parametrize("env,ndev,expect", [
    ({"RANK": "8", "WORLD_SIZE": "16"}, 8, 0),                 # mpirun/srun: no LOCAL_RANK
    ({"RANK": "3", "LOCAL_RANK": "3", "WORLD_SIZE": "4"}, 1, 0),  # one GPU exposed per process
    ({"RANK": "5", "LOCAL_RANK": "5", "LOCAL_WORLD_SIZE": "8", "WORLD_SIZE": "8"}, 8, 5),
])
def test_rccl_init_maps_local_rank_modulo_devices(monkeypatch, env, ndev, expect):
    """Launchers without LOCAL_RANK (it defaults to the global rank) or with one visible GPU per
    process map rank -> device by modulo; only more LOCAL ranks than devices is refused."""
    from distributed_llm_backend_benchmark_amd.parallel import comm as C

    picked = []

    class _Stop(Exception):
        pass

    def _init_pg(**kw):
        raise _Stop()

    monkeypatch.setattr(C.torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(C.torch.cuda, "device_count", lambda: ndev)
    monkeypatch.setattr(C.torch.cuda, "set_device", lambda i: picked.append(i))
    monkeypatch.setattr(C.dist, "is_initialized", lambda: False)
    monkeypatch.setattr(C.dist, "init_process_group", _init_pg)
    for k in ("LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("MASTER_PORT", "1")
    with pytest.raises(_Stop):
        C.init_distributed("rccl")
    assert picked == [expect]


def _agree_worker(rank, world):
    from distributed_llm_backend_benchmark_amd.ops import gemm
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo")
    comm.install_tune_agreement()
    # local timings disagree: alone, rank 0 would pick mfma and rank 1 blas
    local = [{"mfma": 1.0, "blas": 2.0}, {"mfma": 3.0, "blas": 2.5},
             {"mfma": 0.5, "blas": 0.9}, {"mfma": 2.9, "blas": 0.1}][rank]
    best, agreed = gemm._choose(local, "linear", (64, 64, 64))
    mismatch = None
    try:                                   # a rank with another candidate list: refused
        comm.agree_max(["mfma"] if rank == 0 else ["mfma", "pp"], [1.0] * (1 + (rank > 0)))
    except RuntimeError as e:
        mismatch = str(e)
    shape_mismatch = None
    try:                                   # same candidates, different GEMM shape: refused too
        gemm._choose({"mfma": 1.0, "blas": 2.0}, "linear", (64, 64, 64 * (1 + rank)))
    except RuntimeError as e:
        shape_mismatch = str(e)
    comm.destroy()
    alone, _ = (min(local, key=local.get), None)
    return best, agreed, alone, mismatch, gemm._AGREE is None, shape_mismatch


@pytest.mark.parametrize("world", [2, 4])
def test_gemm_autotune_choice_agreed_on_rank_max(world):
    """autotune decisions are collective — every rank takes the argmin of
    the rank-max timings, so ranks with opposite local preferences still run one kernel."""
    res = run_multiprocess(_agree_worker, world)
    bests = {r[0] for r in res}
    assert len(bests) == 1, res
    agreed = res[0][1]
    assert all(r[1] == agreed for r in res)
    assert agreed["mfma"] == max([1.0, 3.0, 0.5, 2.9][:world])
    assert agreed["blas"] == max([2.0, 2.5, 0.9, 0.1][:world])
    assert res[0][2] == "mfma" and res[1][2] == "blas"       # they would have disagreed
    assert all(r[3] and "disagree" in r[3] for r in res)
    assert all(r[4] for r in res)                            # destroy() uninstalls it
    # the tuning key is part of the agreement, a shape mismatch raises everywhere
    assert all(r[5] and "disagree" in r[5] for r in res), [r[5] for r in res]


def test_ddp_tail_bucket_holds_only_late_params_and_split_optimizer_is_exact():
    """the embedding tables (gradient complete only at the end of backward)
    get a bucket of their own, so nothing else waits for the embedding backward; the optimizer
    split around that bucket (AdamW on the other buckets first) is bitwise the single update."""
    from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_llm_backend_benchmark_amd.parallel.ddp import FlatParamTrainer

    cfg = GPT2Config(vocab_size=256, block_size=16, n_layer=3, n_head=2, n_embd=64)
    g = torch.Generator().manual_seed(0)
    idx = torch.randint(0, 256, (2, 17), generator=g)
    finals = {}
    for split in (True, False):
        m = GPT2(cfg, seed=5)
        tr = FlatParamTrainer(m, None, lr=1e-2, bucket_mb=0.05, split_optimizer=split)
        tail = tr.buckets[-1]
        assert {id(p) for p in tail.params} == {id(m.wte), id(m.wpe)}
        assert all(not getattr(p, "_dlbb_late_grad", False)
                   for b in tr.buckets[:-1] for p in b.params)
        assert len(tr.buckets) > 2
        assert tr._split_optimizer_ok() == split
        for _ in range(3):
            tr.step(idx[:, :-1], idx[:, 1:])
        finals[split] = (tr.flat_param.clone(), tr.master.clone(), tr.opt.t)
        tr.close()
    assert torch.equal(finals[True][0], finals[False][0])
    assert torch.equal(finals[True][1], finals[False][1])
    assert finals[True][2] == finals[False][2] == 3


def _run_tp_cli_worker(rank, world, cfg_path, extra):
    from distributed_llm_backend_benchmark_amd.cli import run_tp

    return run_tp.main(["--config", cfg_path, "--backend", "gloo", "--kernels", "torch"] + extra)


def _tiny_tp_config(tmp_path, world):
    import yaml

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = yaml.safe_load(open(os.path.join(repo, "config", "baseline_config.yaml")))
    cfg["model"].update(hidden_size=128, num_layers=2, num_heads=4, ffn_intermediate=512,
                        init_std=0.05)
    cfg["input"].update(batch_size=2, sequence_length=16)
    cfg["execution"].update(warmup_iterations=1, benchmark_iterations=3)
    cfg["parallelism"]["world_size"] = world
    cfg["experiment"]["output_dir"] = str(tmp_path)
    p = tmp_path / "tiny.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return str(p), cfg["experiment"]["name"]


RUN_MPI_KEYS = {"experiment", "backend", "config", "system_info", "rank_0_summary",
                "rank_statistics", "raw_metrics_rank_0"}     # reference run_mpi.py:217-225


def test_run_tp_cli_check_dense_gloo(tmp_path):
    """run_tp at world 2 (gloo): the reference's result schema and the TP output equal to the
    dense model of the same seed (--check-dense), the GEMM-choice agreement recorded."""
    path, name = _tiny_tp_config(tmp_path, 2)
    rc = run_multiprocess(_run_tp_cli_worker, 2, args=(path, ["--check-dense"]))
    assert rc == [0, 0]
    rec = json.load(open(tmp_path / f"gloo_{name}.json"))
    assert RUN_MPI_KEYS <= set(rec)
    assert rec["rank_0_summary"]["world_size"] == 2
    assert rec["throughput"]["dense_check"]["passed"], rec["throughput"]["dense_check"]
    assert rec["throughput"]["gemm_kernel_mix"]["agreed_across_ranks"] is True


def test_run_tp_cli_shard_as(tmp_path):
    """--shard-as P at world 1: rank 0's shard of a P-way model (per-rank shapes, per-rank
    FLOPs), each all-reduce through the local stand-in; the world-size check uses P."""
    path, name = _tiny_tp_config(tmp_path, 4)
    from distributed_llm_backend_benchmark_amd.cli import run_tp

    assert run_tp.main(["--config", path, "--backend", "gloo", "--kernels", "torch",
                        "--shard-as", "4"]) == 0
    rec = json.load(open(tmp_path / f"gloo_{name}_shard4.json"))
    th = rec["throughput"]
    assert th["shard_as"]["P"] == 4
    assert th["allreduce_bytes_per_forward_per_rank"] == 2 * 2 * (2 * 16 * 128 * 2)
    # without --shard-as the same config (world_size 4) is refused at world 1
    assert run_tp.main(["--config", path, "--backend", "gloo", "--kernels", "torch"]) == 1


def _list_allgather_worker(rank, world):
    import torch

    from distributed_llm_backend_benchmark_amd.parallel.collectives import make_data, make_op
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo")
    try:
        res = []
        for n in (1, 7, 4096, 100003):
            x = make_data((n,), torch.bfloat16, rank, comm.device)
            op = make_op("allgather", comm, x, form="list")
            op.run()
            ins = [make_data((n,), torch.bfloat16, r, comm.device) for r in range(world)]
            exact = all(torch.equal(o, i) for o, i in zip(op.outs, ins))
            res.append((n, exact, op.impl))
        return res
    finally:
        comm.destroy()


def test_allgather_list_form_unpack_bit_exact():
    """Reference list form (collectives/1d/dsccl.py:72-76): gathered once into a flat staging
    buffer, unpacked into the list by one chunk-copy table; every entry bit-exact."""
    for rank, res in enumerate(run_multiprocess(_list_allgather_worker, 2, timeout=300)):
        for n, exact, impl in res:
            assert exact, (rank, n)
            assert impl == "allgather_into_tensor+unpack", impl   # recorded as op_impl
