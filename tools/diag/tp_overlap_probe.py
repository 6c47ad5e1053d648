"""Why does the micro-batch interleaved TP forward not hide its all-reduces? (diagnostic)

Rank 0's shard of a P-way 7B TP forward on one GPU (as ``run_tp --shard-as P``), for each
``--chunks`` setting and each comm variant:

* ``none``: every all-reduce skipped (pure compute of that schedule);
* ``reduce``: the stand-in's HBM traffic only;
* ``spin``: only the link-time spin (``--busbw``), no traffic;
* ``both``: what ``run_tp --emulate-busbw`` runs.

Prints one JSON line per (chunks, variant): forward ms (events, mean of ``--iters``), and from
one stamped forward (``utils.stamps``: ping-pong GEMMs, reduction, spin) the comm-busy time, the
GEMM-busy time and how much of the comm-busy time had a GEMM workgroup running beside it.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def _union(intervals):
    out = []
    for a, b in sorted(intervals):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _overlap(u1, u2):
    i = j = 0
    tot = 0.0
    while i < len(u1) and j < len(u2):
        a, b = max(u1[i][0], u2[j][0]), min(u1[i][1], u2[j][1])
        if b > a:
            tot += b - a
        if u1[i][1] < u2[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--chunks", default="1,2")
    ap.add_argument("--variants", default="none,reduce,spin,both")
    ap.add_argument("--busbw", type=float, default=300.0)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--streams", default="1", help="chunk_streams settings to run (0,1)")
    ap.add_argument("--pg-eager", action="store_true",
                    help="with --init-pg: eager communicator init (device_id=, as "
                         "parallel.comm.init_distributed does)")
    ap.add_argument("--init-pg", action="store_true",
                    help="first bring up a world-1 RCCL process group and run one all-reduce "
                         "(as run_tp does), to see what its streams do to the overlap")
    args = ap.parse_args()

    import torch

    if args.init_pg:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        torch.cuda.set_device(0)
        kw = {"device_id": torch.device("cuda", 0)} if args.pg_eager else {}
        dist.init_process_group("nccl", rank=0, world_size=1, **kw)
        if not args.pg_eager:
            t = torch.ones(1024, device="cuda")
            dist.all_reduce(t)
        torch.cuda.synchronize()

    from distributed_llm_backend_benchmark_amd.models.tp_transformer import LLM
    from distributed_llm_backend_benchmark_amd.ops.elementwise import spin_ns
    from distributed_llm_backend_benchmark_amd.parallel.comm import Comm
    from distributed_llm_backend_benchmark_amd.parallel.tensor_parallel import RowParallelLinear
    from distributed_llm_backend_benchmark_amd.utils.stamps import Stamps

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm(rank=0, world_size=args.P, local_rank=0, backend="emulate", device=dev)
    x = torch.randn(8, 512, 4096, device=dev).to(torch.bfloat16)
    cfgs = []
    for n in [int(c) for c in args.chunks.split(",")]:
        for cs in ([1] if n == 1 else [int(v) for v in args.streams.split(",")]):
            cfgs.append((n, cs))
    for n, cs in cfgs:
        model = LLM(hidden_size=4096, num_layers=args.layers, num_heads=32,
                    ffn_intermediate=16384, comm=comm, seed=42, allreduce="emulate",
                    overlap_chunks=n)
        model.chunk_streams = bool(cs)
        rows = [m for m in model.modules() if isinstance(m, RowParallelLinear)]
        for variant in args.variants.split(","):
            for m in rows:
                m.emulate_busbw = args.busbw if variant in ("spin", "both") else None
                if variant == "none":
                    m._all_reduce = lambda t: None
                elif variant == "spin":
                    P = args.P

                    def spin_only(t, m=m, P=P):
                        nb = t.numel() * t.element_size()
                        spin_ns(int(nb * 2.0 * (P - 1) / P / args.busbw), m.emulate_blocks,
                                t.device)
                    m._all_reduce = spin_only
                else:
                    m.__dict__.pop("_all_reduce", None)
            with torch.no_grad():
                for _ in range(3):
                    model(x)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                import time as _time

                issue = []
                e0.record()
                for _ in range(args.iters):
                    t0 = _time.perf_counter()
                    model(x)
                    issue.append(_time.perf_counter() - t0)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.iters
                with Stamps(1 << 21) as st:
                    model(x)
                launches = st.collect()
            comm_iv = [(a, b) for L in launches if L["kind"] in ("spin", "reduce_sum")
                       for a, b in zip(L["start_ns"], L["end_ns"])]
            gemm_iv = [(a, b) for L in launches if L["kind"].startswith("gemm")
                       for a, b in zip(L["start_ns"], L["end_ns"])]
            uc, ug = _union(comm_iv), _union(gemm_iv)
            busy_c = sum(b - a for a, b in uc)
            busy_g = sum(b - a for a, b in ug)
            span = (max(b for _, b in comm_iv + gemm_iv) - min(a for a, _ in comm_iv + gemm_iv)
                    if comm_iv or gemm_iv else 0.0)
            print(json.dumps({
                "P": args.P, "chunks": n, "chunk_streams": bool(cs), "variant": variant,
                "busbw": args.busbw, "init_pg": args.init_pg, "pg_eager": args.pg_eager,
                "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                "forward_ms": round(ms, 3), "stamped_launches": len(launches),
                "host_issue_ms": round(1e3 * sorted(issue)[len(issue) // 2], 3),
                "cpu_affinity": len(os.sched_getaffinity(0)),
                "stamped_span_ms": round(span / 1e6, 3),
                "comm_busy_ms": round(busy_c / 1e6, 3), "gemm_busy_ms": round(busy_g / 1e6, 3),
                "comm_under_gemm_ms": round(_overlap(uc, ug) / 1e6, 3),
                "gemm_launches": sum(1 for L in launches if L["kind"].startswith("gemm")),
            }), flush=True)
        del model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
