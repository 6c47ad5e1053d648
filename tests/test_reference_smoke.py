"""The reference's smoke-test checks, as pytest over Gloo processes on localhost.

Reference: ``test/test_open.py`` (mpi4py, 12 checks at :17-271: p2p, bcast, scatter, gather,
allgather, reduce, allreduce, buffer Bcast/Allreduce, barrier with staggered sleep, ring
isend/irecv, MAX/MIN/PROD) and ``test/test_deepseed.py`` (torch.distributed ccl, 8 checks at
:31-181). The reference needs mpirun/deepspeed and aborts the communicator on failure
(``test/test_open.py:329``); here each check is an assertion inside a spawned rank and the
parent reports the failing rank.
"""

import time

import pytest
import torch

from mp_utils import run_multiprocess


def _checks(rank, world):
    import torch.distributed as dist

    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("gloo")
    out = {}
    # point-to-point (test_open.py:35-63): rank 0 sends a payload to every other rank
    if rank == 0:
        for r in range(1, world):
            dist.send(torch.tensor([42.0, float(r)]), dst=r)
    else:
        t = torch.empty(2)
        dist.recv(t, src=0)
        assert t.tolist() == [42.0, float(rank)]
    out["p2p"] = True
    # broadcast (:65-84)
    t = torch.arange(4, dtype=torch.float32) if rank == 0 else torch.zeros(4)
    dist.broadcast(t, src=0)
    assert t.tolist() == [0.0, 1.0, 2.0, 3.0]
    # scatter (:86-103)
    o = torch.zeros(2)
    dist.scatter(o, [torch.full((2,), float(r * 10)) for r in range(world)] if rank == 0 else None,
                 src=0)
    assert o.tolist() == [rank * 10.0] * 2
    # gather (:105-123)
    gl = [torch.zeros(1) for _ in range(world)] if rank == 0 else None
    dist.gather(torch.tensor([float(rank)]), gl, dst=0)
    if rank == 0:
        assert [x.item() for x in gl] == [float(r) for r in range(world)]
    # allgather (:125-140)
    al = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(al, torch.tensor([float(rank * rank)]))
    assert [x.item() for x in al] == [float(r * r) for r in range(world)]
    # reduce (:142-157)
    t = torch.tensor([float(rank + 1)])
    dist.reduce(t, dst=0)
    if rank == 0:
        assert t.item() == world * (world + 1) / 2
    # allreduce (:159-173)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    assert t.item() == world * (world + 1) / 2
    # buffer Bcast / Allreduce of an array (:175-212)
    arr = torch.arange(1000, dtype=torch.float64) * (rank + 1)
    dist.all_reduce(arr)
    assert torch.equal(arr, torch.arange(1000, dtype=torch.float64) * world * (world + 1) / 2)
    # barrier with staggered arrival (:214-225)
    t0 = time.time()
    time.sleep(0.05 * rank)
    comm.barrier()
    assert time.time() - t0 >= 0.05 * (world - 1) - 0.01
    # ring isend/irecv (:227-246)
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    recv = torch.zeros(3)
    reqs = [dist.isend(torch.full((3,), float(rank)), nxt), dist.irecv(recv, prv)]
    for q in reqs:
        q.wait()
    assert recv.tolist() == [float(prv)] * 3
    # MAX / MIN / PROD (:248-271; test_deepseed.py all_reduce MAX :158-176)
    for op, want in ((dist.ReduceOp.MAX, float(world)), (dist.ReduceOp.MIN, 1.0),
                     (dist.ReduceOp.PRODUCT, float(torch.arange(1, world + 1).prod()))):
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t, op=op)
        assert t.item() == want, (op, t.item(), want)
    # object collectives (mpi4py lower-case pickle path: 1d/openmpi.py:63,78,113)
    objs = comm.all_gather_object({"rank": rank, "msg": f"hello from {rank}"})
    assert [o["rank"] for o in objs] == list(range(world))
    assert comm.broadcast_object({"cfg": [1, 2, 3]} if rank == 0 else None) == {"cfg": [1, 2, 3]}
    # timing side channel: uneven per-rank lists gathered as [rank][iter]
    g = comm.gather_floats([0.5] * (rank + 1))
    if rank == 0:
        assert [len(x) for x in g] == [r + 1 for r in range(world)]
    comm.destroy()
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_reference_smoke_checks(world):
    res = run_multiprocess(_checks, world, timeout=240)
    assert all(r["p2p"] for r in res)


def test_world_size_mismatch_exits(tmp_path):
    """run_mpi.py:73-77: a config asking for a different world size exits with status 1."""
    import subprocess
    import sys

    import yaml

    from conftest import REPO

    cfg = yaml.safe_load(open(f"{REPO}/config/baseline_config.yaml"))
    cfg["model"].update(hidden_size=64, num_layers=1, num_heads=2, ffn_intermediate=128)
    cfg["input"].update(batch_size=1, sequence_length=8)
    cfg["parallelism"]["world_size"] = 3
    cfg["experiment"]["output_dir"] = str(tmp_path)
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([sys.executable, "-m", "distributed_llm_backend_benchmark_amd.cli.run_tp",
                        "--config", str(p), "--backend", "gloo"], cwd=REPO, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 1 and "World size mismatch" in r.stdout
    cfg["parallelism"]["world_size"] = 1
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([sys.executable, "-m", "distributed_llm_backend_benchmark_amd.cli.run_tp",
                        "--config", str(p), "--backend", "gloo", "--iters", "2", "--warmup", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    import json

    res = json.load(open(tmp_path / "gloo_baseline_7b_world4.json"))
    assert set(res) >= {"experiment", "backend", "config", "system_info", "rank_0_summary",
                        "rank_statistics", "raw_metrics_rank_0"}
    assert res["rank_0_summary"]["num_iterations"] == 2
