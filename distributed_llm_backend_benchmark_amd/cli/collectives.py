"""Collective sweep CLI — every constant the reference hard-codes is a flag.

Reference drivers: ``collectives/1d/{openmpi,intelmpi,dsccl,dsgloo}.py`` (constants at
``1d/openmpi.py:13-49``) and ``collectives/3d/*.py`` (constants at ``3d/openmpi.py:16-35``,
``3d/dsccl.py:16-32``). One driver replaces all of them; the backend is the process group.

Examples (one process per GPU)::

    # reference 1D sweep: 8 ops x {1KB,64KB,1MB,16MB}, 10 warmup / 100 timed
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m \
        distributed_llm_backend_benchmark_amd.cli.collectives --mode 1d
    # full power-of-two sweep 1 KiB .. 1 GiB, all-reduce only, nccl-tests style batches too
    ... --mode 1d --ops allreduce --sizes sweep --batched --graph
    # 3D activation grid (reference BATCH x SEQ x HIDDEN), fp32-on-wire variant
    ... --mode 3d --ops allreduce,allgather,reduce_scatter --wire-dtype fp32
    # RCCL algorithm variant (analogue of CCL_ALLREDUCE=ring, 3d/launch_dsccl.sh:46-47)
    ... --mode 3d --ops allreduce --env NCCL_ALGO=Ring --impl-name rccl_ring_allreduce
    # IPC one-shot / two-shot xGMI kernel instead of RCCL
    ... --mode 1d --ops allreduce --allreduce-impl custom --impl-name custom_allreduce
"""

from __future__ import annotations

import argparse
import os
import sys


def _ints(s: str):
    return [int(x) for x in s.split(",") if x.strip()]


def parse_args(argv=None):
    from ..parallel.collectives import REFERENCE_1D_OPS, REFERENCE_3D_OPS  # noqa: F401

    ap = argparse.ArgumentParser(description="MI355X collective sweep (RCCL over xGMI / Gloo)")
    ap.add_argument("--mode", choices=["1d", "3d"], default="1d")
    ap.add_argument("--backend", default="auto", choices=["auto", "rccl", "gloo"])
    ap.add_argument("--ops", default=None,
                    help="comma list; default = the reference's op list for the mode "
                         "(+ reduce_scatter for 3d)")
    ap.add_argument("--sizes", default="reference",
                    help="1D: reference | sweep | LO:HI (e.g. 1KiB:4GiB) | comma list")
    ap.add_argument("--batch-sizes", default="1,8,16,32")
    ap.add_argument("--seq-lengths", default="1,2048,4096,8192")
    ap.add_argument("--hidden-dims", default="2048,4096")
    ap.add_argument("--dtype", default=None, help="bf16 | fp16 | fp32 (default fp16 1D, bf16 3D)")
    ap.add_argument("--wire-dtype", default=None, help="3D: cast to this dtype before the op")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--output-dir", default=None)
    ap.add_argument("--impl-name", default=None, help="implementation label in names/JSON")
    ap.add_argument("--timing", default="auto", choices=["auto", "hip_event", "host"])
    ap.add_argument("--batched", action="store_true", help="also time back-to-back calls")
    ap.add_argument("--graph", action="store_true", help="capture the batched loop in a HIP graph")
    ap.add_argument("--validate", action="store_true", help="check results against closed forms")
    ap.add_argument("--resume", action="store_true", help="skip configs whose JSON exists")
    ap.add_argument("--allreduce-impl", default="rccl", choices=["rccl", "custom", "auto"])
    ap.add_argument("--engine", default="torch", choices=["torch", "native"],
                    help="torch = collectives through torch.distributed (ProcessGroupNCCL); "
                         "native = our C++ RCCL engine enqueuing on the timing stream")
    ap.add_argument("--allreduce-algo", default=None, choices=["oneshot", "twoshot"])
    ap.add_argument("--direct-ipc", action="store_true",
                    help="allgather / reduce_scatter / alltoall through the direct one-hop IPC "
                         "kernels (each GPU pulls from all peers over its xGMI links) instead "
                         "of RCCL")
    ap.add_argument("--allgather-form", default="tensor", choices=["tensor", "list"])
    ap.add_argument("--env", action="append", default=[],
                    help="KEY=VAL exported before the process group starts (RCCL knobs: "
                         "NCCL_ALGO, NCCL_PROTO, NCCL_MIN_NCHANNELS, NCCL_MAX_NCHANNELS, ...)")
    ap.add_argument("--trace", action="store_true",
                    help="emit roctx ranges (record with rocprofv3 --marker-trace)")
    ap.add_argument("--torch-profile", default=None, metavar="DIR",
                    help="torch.profiler Chrome trace per rank into DIR")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--timeout", type=float, default=900.0, help="process-group timeout (s)")
    ap.add_argument("--device", choices=["auto", "cpu", "cuda"], default="auto",
                    help="tensor device; auto = cuda for rccl, cpu for gloo. gloo + cuda = ranks "
                         "sharing one GPU over a gloo process group (rehearsal of the multi-rank "
                         "sweep; RCCL needs one GPU per rank)")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    env = {}
    for kv in args.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
        env[k] = v

    from ..bench import schema
    from ..bench.sweep import run_1d_sweep, run_3d_sweep
    from ..parallel.collectives import REFERENCE_1D_OPS, REFERENCE_3D_OPS
    from ..parallel.comm import init_distributed

    comm = init_distributed(args.backend, timeout_s=args.timeout,
                            device=None if args.device == "auto" else args.device)
    impl = args.impl_name or comm.backend_label
    if args.ops:
        ops = [o.strip() for o in args.ops.split(",") if o.strip()]
    else:
        ops = list(REFERENCE_1D_OPS) if args.mode == "1d" else list(REFERENCE_3D_OPS) + [
            "reduce_scatter", "alltoall"]
    op_opts = {"impl": "native" if args.engine == "native" else args.allreduce_impl,
               "form": args.allgather_form, "direct": args.direct_ipc}
    if args.allreduce_algo:
        op_opts["algo"] = 1 if args.allreduce_algo == "oneshot" else 2
    extra = {"env": env} if env else {}
    extra["engine"] = args.engine
    if comm.is_gpu:
        import torch

        extra["device"] = torch.cuda.get_device_name(comm.device)
    outdir = args.output_dir or os.path.join("results", args.mode, impl)
    from ..utils import tracing

    if args.trace:
        tracing.enable()
    timing = args.timing if args.timing != "host" else "host_perf_counter"
    try:
        with tracing.torch_profile(args.torch_profile, comm.rank):
            if args.mode == "1d":
                dtype = args.dtype or "fp16"
                elem = 4 if dtype in ("fp32", "float32") else 2
                sizes = schema.resolve_1d_sizes(args.sizes, elem)
                run_1d_sweep(comm, ops=ops, sizes=sizes, dtype=dtype, warmup=args.warmup,
                             iters=args.iters, output_dir=outdir, impl_name=impl,
                             timing=timing,
                             batched=args.batched, graph=args.graph, validate=args.validate,
                             resume=args.resume, seed=args.seed, op_opts=op_opts, extra=extra)
            else:
                run_3d_sweep(comm, ops=ops, batch_sizes=_ints(args.batch_sizes),
                             seq_lengths=_ints(args.seq_lengths),
                             hidden_dims=_ints(args.hidden_dims),
                             dtype=args.dtype or "bf16", wire_dtype=args.wire_dtype,
                             warmup=args.warmup, iters=args.iters, output_dir=outdir,
                             impl_name=impl,
                             timing=timing,
                             batched=args.batched, graph=args.graph, validate=args.validate,
                             resume=args.resume, seed=args.seed, op_opts=op_opts, extra=extra)
    finally:
        comm.barrier()
        comm.destroy()
    if comm.rank == 0:
        print(f"Results saved in '{outdir}/'")
    return 0


if __name__ == "__main__":
    sys.exit(main())
