"""GPT-2-small DDP training microbenchmark (BASELINE config 5).

Each rank trains the same GPT-2 on its own synthetic token batch; gradients are bucketed
(contiguous slices of one flat bf16 gradient buffer) and all-reduced over RCCL while backward is
still running (:mod:`..parallel.ddp`), then one fused AdamW kernel updates the fp32 masters and
the bf16 working weights. Reported: tokens/s over the whole job (weak scaling: fixed
micro-batch per GPU), ms/step (max over ranks), model TFLOP/s per GPU, and the same step with
overlap disabled for comparison (``--compare-overlap``).

Launch::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m \
        distributed_llm_backend_benchmark_amd.cli.train_ddp --batch 16 --seq 1024
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="GPT-2 DDP training microbenchmark")
    ap.add_argument("--backend", default="auto", choices=["auto", "rccl", "gloo"])
    ap.add_argument("--n-layer", type=int, default=12)
    ap.add_argument("--n-head", type=int, default=12)
    ap.add_argument("--n-embd", type=int, default=768)
    ap.add_argument("--vocab", type=int, default=50304)
    ap.add_argument("--batch", type=int, default=16, help="micro-batch per GPU")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--lr-warmup", type=int, default=10,
                    help="linear learning-rate warmup over the first N optimizer steps (Adam "
                         "without warmup can spike on this synthetic data); under --graph the "
                         "rate is the one in effect at capture")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--mode", choices=["view", "flatten"], default="view")
    ap.add_argument("--allreduce", choices=["auto", "rccl", "custom", "native"], default="auto",
                    help="bucket all-reduce. auto (default): registered in-place IPC xGMI kernel "
                         "for buckets up to the node-calibrated crossover, our C++ RCCL engine "
                         "above it, both on a probed comm stream. rccl: torch ProcessGroupNCCL "
                         "(A/B only: its internal pool stream can share the compute stream's "
                         "hardware queue and serialise backward with comm, parallel/streams.py). "
                         "custom: IPC kernel for every bucket. native: C++ RCCL engine for every "
                         "bucket")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--comm-blocks", type=int, default=None,
                    help="CU budget: workgroups per bucket-reduction launch (IPC kernel / "
                         "emulation); default = the kernel's size heuristic")
    ap.add_argument("--emulate-comm", nargs="?", const=True, default=False, type=float,
                    metavar="BUSBW_GBPS",
                    help="world 1: run a bucket-sized stand-in reduction (one rank's all-reduce "
                         "HBM traffic) on the comm stream at every bucket-ready hook, to measure "
                         "what overlapped gradient reduction costs the backward pass; with a "
                         "value, each stand-in also lasts the ring all-reduce time at that bus "
                         "bandwidth over --emulate-world ranks (link-bound)")
    ap.add_argument("--emulate-world", type=int, default=8)
    ap.add_argument("--no-late-bucket", action="store_true",
                    help="A/B: do not give the embedding tables a bucket of their own")
    ap.add_argument("--no-split-optimizer", action="store_true",
                    help="A/B: one AdamW pass after every bucket is reduced")
    ap.add_argument("--comm-timeline", action="store_true",
                    help="after the timed steps, one more step with comm events: bytes reduced "
                         "after backward and the exposed comm time (stream-issued reductions)")
    ap.add_argument("--zero", action="store_true",
                    help="ZeRO-2-style: reduce-scatter grads, sharded AdamW, all-gather params")
    ap.add_argument("--compare-overlap", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step in a HIP graph after warmup and replay "
                         "it (world 1, or --allreduce native|custom)")
    ap.add_argument("--save-checkpoint", default=None, metavar="DIR",
                    help="after the timed steps, write master weights + AdamW state (safetensors)")
    ap.add_argument("--resume-from", default=None, metavar="DIR",
                    help="load a checkpoint written by --save-checkpoint before warmup")
    ap.add_argument("--trace", action="store_true",
                    help="emit roctx ranges (record with rocprofv3 --marker-trace)")
    ap.add_argument("--torch-profile", default=None, metavar="DIR",
                    help="torch.profiler Chrome trace per rank into DIR")
    ap.add_argument("--main-stream-priority", type=int, default=0, choices=[0, -1],
                    help="-1: run the step on a HIGH-priority stream, so the critical-path "
                         "kernels are dispatched ahead of the side-stream weight gradients / "
                         "bucket reductions (A/B)")
    ap.add_argument("--output", default=None, help="write the result JSON here (rank 0)")
    return ap.parse_args(argv)


def _path_counts(tr) -> dict:
    paths = tr.bucket_paths() if hasattr(tr, "bucket_paths") else {}
    out = {}
    for p in paths.values():
        out[p] = out.get(p, 0) + 1
    return out


def _stream_roles(tr, comm) -> dict:
    """hipStream_t handles of the step's streams by role, plus every probed candidate, so a
    rocprofv3 kernel trace (Stream_Id / Queue_Id per dispatch) can be read by role."""
    if not comm.is_gpu:
        return {}
    import torch

    from ..parallel import streams as S

    def h(s):
        return hex(s.cuda_stream) if s is not None else None
    return {"compute": h(torch.cuda.current_stream(comm.device)),
            "wgrad": [h(s) for s in getattr(tr, "_wgrad_streams", []) or []],
            "comm": h(getattr(tr, "_comm_stream", None)),
            "opt": h(getattr(tr, "_opt_stream", None)),
            "probed": list(S.LOG)}


def run(args, comm, overlap: bool):
    import torch

    from ..models.gpt2 import GPT2, GPT2Config
    from ..parallel.ddp import FlatParamTrainer

    cfg = GPT2Config(vocab_size=args.vocab, block_size=args.seq, n_layer=args.n_layer,
                     n_head=args.n_head, n_embd=args.n_embd)
    model = GPT2(cfg, device=comm.device)
    if args.zero:
        from ..parallel.zero import ShardedTrainer

        tr = ShardedTrainer(model, comm, lr=args.lr, bucket_mb=args.bucket_mb, overlap=overlap)
    else:
        tr = FlatParamTrainer(model, comm if comm.world_size > 1 else None, lr=args.lr,
                              bucket_mb=args.bucket_mb, overlap=overlap, mode=args.mode,
                              allreduce=args.allreduce, comm_blocks=args.comm_blocks,
                              emulate_comm=args.emulate_comm, emulate_world=args.emulate_world,
                              late_bucket=not args.no_late_bucket,
                              split_optimizer=not args.no_split_optimizer)
    # everything after the trainer registered its buckets runs under try/finally, so
    # a failure (an agreed one: check_comm_errors, a section's candidate) still releases the IPC
    # registrations and gradient buffers before the caller moves on to the next candidate
    try:
        return _train(args, comm, tr, model, cfg)
    finally:
        tr.close()
        del tr, model
        if comm.is_gpu:
            torch.cuda.empty_cache()


def _train(args, comm, tr, model, cfg):
    from ..data import SyntheticTokenDataset

    data = SyntheticTokenDataset(args.batch, args.seq, cfg.vocab_size, rank=comm.rank,
                                 device=comm.device)
    if args.resume_from:
        tr.load_checkpoint(args.resume_from)

    def set_lr():   # host-side scalar: one attribute per step, no device work
        tr.opt.lr = args.lr * min(1.0, (tr.step_count + 1) / max(1, args.lr_warmup))

    first_loss = None
    for i in range(args.warmup):
        x, y = data.get_batch()
        set_lr()
        out = tr.step(x, y, sync_loss=(i == 0))
        if i == 0:
            first_loss = out

    def step_fn(x, y):
        set_lr()
        return tr.step(x, y, sync_loss=False)
    if hasattr(tr, "recheck_side_streams"):
        tr.recheck_side_streams()       # after warm-up, outside the timed steps
    if args.graph:
        x, y = data.get_batch()
        step_fn = tr.capture_step(x, y)
    comm.barrier()
    comm.sync()
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        x, y = data.get_batch()
        loss = step_fn(x, y)
    comm.sync()
    dt = comm.allreduce_max(time.perf_counter() - t0)
    tr.check_comm_errors()              # collective; raises on every rank after an IPC timeout
    from ..ops import gemm as _gemm

    res = {
        "ms_per_step": dt / args.steps * 1e3,
        "tokens_per_s": comm.world_size * args.batch * args.seq * args.steps / dt,
        "loss": float(loss.item()) if loss is not None else None,
        "loss_first_step": first_loss,
        "params": model.num_parameters(),
        "buckets": len(tr.buckets),
        "hip_graph": bool(args.graph),
        "tflops_per_gpu": model.flops_per_token(args.seq) * args.batch * args.seq
        * args.steps / dt / 1e12,
        "gemm_kernel_mix": _gemm.kernel_mix(),
        # node-measured IPC-vs-RCCL crossovers (rank-max, agreed; None: no IPC kernel)
        "allreduce_calibration": getattr(getattr(tr, "_car", None), "calibration", None),
        # which all-reduce each bucket took (auto picks per bucket size)
        "bucket_paths": _path_counts(tr),
        "gemm_tune_timing": _gemm.tune_timing(),
        # per-bucket AdamW during backward (parallel/ddp.py _OPT_OVERLAP; 0 = after backward)
        "opt_overlap": getattr(tr, "opt_overlap", 0),
        "side_stream_checks": getattr(tr, "side_stream_checks", []),
        "streams": _stream_roles(tr, comm),
    }
    if args.comm_timeline and not args.zero:
        tr.timeline = True
        x, y = data.get_batch()
        set_lr()
        tr.step(x, y, sync_loss=False)
        tr.timeline = False
        res["comm_tail"] = tr.comm_tail_report()
    if args.save_checkpoint:
        tr.save_checkpoint(args.save_checkpoint)
        res["checkpoint"] = args.save_checkpoint
    res["step_count"] = tr.step_count
    return res


def main(argv=None) -> int:
    args = parse_args(argv)
    from ..parallel.comm import init_distributed

    from ..utils import tracing

    comm = init_distributed(args.backend, timeout_s=900)
    comm.install_tune_agreement()       # GEMM kernel choices agreed on rank-max timings
    affinity = comm.affinity_all_ranks()    # host threads on the GPU's NUMA node (collective)
    if args.trace:
        tracing.enable()
    import contextlib

    import torch

    main_ctx = contextlib.nullcontext()
    if args.main_stream_priority and comm.is_gpu:
        main_ctx = torch.cuda.stream(torch.cuda.Stream(comm.device,
                                                       priority=args.main_stream_priority))
    with tracing.torch_profile(args.torch_profile, comm.rank), main_ctx:
        main_res = run(args, comm, overlap=not args.no_overlap)
    out = {"metric": "gpt2_ddp_tokens_per_s", "value": main_res["tokens_per_s"],
           "n_gpus": comm.world_size, "overlap": not args.no_overlap, **main_res,
           "host_affinity_per_rank": affinity,
           "config": {k: getattr(args, k) for k in ("n_layer", "n_head", "n_embd", "vocab",
                                                    "batch", "seq", "bucket_mb", "mode",
                                                    "allreduce", "zero", "comm_blocks",
                                                    "emulate_comm", "emulate_world",
                                                    "no_late_bucket",
                                                    "no_split_optimizer",
                                                    "main_stream_priority")}}
    if args.compare_overlap:
        alt = run(args, comm, overlap=args.no_overlap)
        out["other_overlap_setting"] = alt
    if comm.rank == 0:
        print(json.dumps(out), flush=True)
        if args.output:
            os.makedirs(os.path.dirname(os.path.abspath(args.output)), exist_ok=True)
            with open(args.output, "w") as f:
                json.dump(out, f, indent=2)
    comm.barrier()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
