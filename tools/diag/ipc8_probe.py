"""Diagnostic: where does the 8-ranks-on-one-GPU direct IPC test spend its
time? Runs the FULL matrix of ``tests/test_comm_gpu.py::_direct_worker`` (all-gather /
reduce-scatter / all-to-all x bf16 / fp32 x nblocks None / 3 / 256, 3 calls each, then the uneven
MoE all-to-all at nblocks None / 5 / 256) with every rank appending one JSON line per call to
``<out>/rank<r>.jsonl`` as soon as the call has completed on the device: host wall time of the
launch, of the synchronize, the device-side timeout flag, and the number of HIP streams the rank
has touched. Lines are flushed per call, so a stall shows which call, on which rank, and whether
the host was inside the launch or inside the synchronize.

Usage: ``python tools/diag/ipc8_probe.py <out_dir> [world] [hw_queues|default]``.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "tests"))


def worker(rank, world, out_dir):
    import torch

    from distributed_llm_backend_benchmark_amd.parallel.collectives import make_data, make_op
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    f = open(os.path.join(out_dir, f"rank{rank}.jsonl"), "w")
    t_origin = time.time()

    def log(**kw):
        kw["t"] = round(time.time() - t_origin, 4)
        f.write(json.dumps(kw) + "\n")
        f.flush()

    log(ev="start", pid=os.getpid(), hwq=os.environ.get("GPU_MAX_HW_QUEUES", "default"))
    comm = init_distributed("gloo", device="cuda")
    log(ev="init_done")
    n = world * 8 * 1000
    ok_all = True
    for dt in (torch.bfloat16, torch.float32):
        ins = [make_data((n,), dt, r, torch.device("cuda")) for r in range(world)]
        for name in ("allgather", "reduce_scatter", "alltoall"):
            for nb in (None, 3, 256):
                t0 = time.perf_counter()
                op = make_op(name, comm, ins[rank], direct=True, nblocks=nb)
                t_reg = time.perf_counter() - t0
                for call in range(3):
                    op.reset()
                    t0 = time.perf_counter()
                    op.run()
                    t1 = time.perf_counter()
                    torch.cuda.synchronize()
                    t2 = time.perf_counter()
                    log(op=name, dt=str(dt)[6:], nb=nb, call=call, reg_s=round(t_reg, 4),
                        launch_ms=round((t1 - t0) * 1e3, 3), sync_ms=round((t2 - t1) * 1e3, 3))
                ok = bool(op.check(ins))
                ok_all &= ok
                log(op=name, dt=str(dt)[6:], nb=nb, ev="checked", ok=ok, impl=op.impl)
    for hidden in (1024, 8):
        ins = [make_data((2000, hidden), torch.bfloat16, r, torch.device("cuda"))
               for r in range(world)]
        for nb in (None, 5, 256):
            op = make_op("alltoall_moe", comm, ins[rank], direct=True, nblocks=nb)
            for call in range(3):
                t0 = time.perf_counter()
                op.run()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                log(op="alltoall_moe", h=hidden, nb=nb, call=call,
                    launch_ms=round((t1 - t0) * 1e3, 3), sync_ms=round((t2 - t1) * 1e3, 3))
            exact = torch.equal(op.result().float(), op.expected(ins))
            ok_all &= bool(exact)
            log(op="alltoall_moe", h=hidden, nb=nb, ev="checked", ok=bool(exact))
            op.close()
    comm.barrier()
    log(ev="done", ok=ok_all)
    comm.destroy()
    f.close()
    return ok_all


def main():
    out_dir = sys.argv[1]
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    q = sys.argv[3] if len(sys.argv) > 3 else "default"
    os.makedirs(out_dir, exist_ok=True)
    if q != "default":
        os.environ["GPU_MAX_HW_QUEUES"] = q
    else:
        os.environ.pop("GPU_MAX_HW_QUEUES", None)
    from mp_utils import run_multiprocess
    t0 = time.time()
    res = run_multiprocess(worker, world, args=(out_dir,), timeout=200, hw_queues=None)
    print(json.dumps({"world": world, "hw_queues": q, "ok": all(res),
                      "wall_s": round(time.time() - t0, 2)}), flush=True)


if __name__ == "__main__":
    main()
