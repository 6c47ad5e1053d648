"""The multi-process launchers cannot lose a port race: a port somebody
else holds does not fail the launch, and the spawned-worker harness binds no port in workers."""

import os
import socket

from launch_utils import REPO, run_torchrun
from mp_utils import run_multiprocess

PROBE = os.path.join(REPO, "tests", "scripts", "allreduce_probe.py")


def test_torchrun_survives_a_taken_port():
    """Hold the first chosen port bound and listening: the static launch fails on EADDRINUSE and
    the launcher is started again in the standalone form, which binds port 0 itself."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        s.listen(1)
        taken = s.getsockname()[1]
        env = {k: v for k, v in os.environ.items() if k != "CUDA_VISIBLE_DEVICES"}
        out = run_torchrun(2, [PROBE], 180, env=env, port=taken)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("allreduce_probe")]
    assert len(lines) == 2 and all(l.endswith(" 3.0") for l in lines), out.stdout
    assert all(f"port {taken} " not in l for l in lines), lines


def _sum_worker(rank, world):
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    dist.destroy_process_group()
    return t.item()


def test_spawned_workers_join_a_parent_held_store():
    assert run_multiprocess(_sum_worker, 2, timeout=120) == [3.0, 3.0]
