"""Multi-process helpers for CPU (gloo) and single-GPU multi-rank tests."""

import os
import traceback

import torch.multiprocessing as mp


def _entry(rank, world, port, fn, args, q):
    # the parent holds the TCPStore server (hold_store, bound on port 0): every rank joins it as
    # a client, so no worker binds a port and there is no free-port race
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", TORCHELASTIC_USE_AGENT_STORE="True")
    try:
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
    except BaseException as e:  # report to parent
        q.put((rank, "err", f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))


def run_multiprocess(fn, world, args=(), timeout=240, hw_queues=None):
    """Run ``fn(rank, world, *args)`` in ``world`` spawned processes; returns results by rank.
    ``hw_queues``: None = inherit the environment (HIP's default 4 hardware queues per process);
    "auto" = the round-4 cap of 2 queues per rank at 8+ ranks (kept only for A/B runs: the
    8-rank slowness it was added for was the gloo-leg calibration, see custom_allreduce)."""
    from launch_utils import hold_store

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = hold_store(world)
    port = store.port
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    old_q = os.environ.get("GPU_MAX_HW_QUEUES")
    cap = hw_queues == "auto" and world >= 8 and old_q is None
    if cap:
        os.environ["GPU_MAX_HW_QUEUES"] = "2"
    try:
        for p in procs:
            p.start()
    finally:
        if cap:
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
    out = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        del store
    return [out[r] for r in range(world)]
