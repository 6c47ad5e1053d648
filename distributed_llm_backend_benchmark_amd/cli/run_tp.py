"""Tensor-parallel transformer forward benchmark — ``run_mpi.py`` parity.

Reference: ``run_mpi.py:52-248`` (argparse ``--config``/``--backend``; world-size check;
init timing; warmup loop; timed loop with a barrier before and after each forward; per-rank
forward means gathered to rank 0 with variance / CV; JSON ``{output_dir}/{backend}_{name}.json``
with keys ``experiment, backend, config, system_info, rank_0_summary, rank_statistics,
raw_metrics_rank_0`` (``run_mpi.py:217-225``)).

Launch (one process per GPU)::

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m \
        distributed_llm_backend_benchmark_amd.cli.run_tp --config config/baseline_config.yaml \
        --backend rccl

Differences by design: the forward is device-timed (barrier, then synchronised wall clock and
HIP events); ``--backend`` picks the process-group backend (``rccl`` | ``gloo``) and names the
output file; extra result keys: ``tokens_per_s``, ``tflops_per_rank``, ``allreduce_bytes``.
"""

from __future__ import annotations

import argparse
import os
import sys
import time


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="TP transformer forward benchmark (run_mpi.py parity)")
    ap.add_argument("--config", required=True, help="YAML config (reference schema)")
    ap.add_argument("--backend", default="rccl", choices=["rccl", "gloo", "nccl"],
                    help="process-group backend; also names the output file")
    ap.add_argument("--allreduce", choices=["auto", "rccl", "custom", "native"], default=None,
                    help="override execution.allreduce")
    ap.add_argument("--device", choices=["auto", "cpu", "cuda"], default="auto",
                    help="tensor device; auto = cuda for rccl, cpu for gloo. gloo + cuda = "
                         "several ranks sharing one GPU over a gloo process group (rehearsal "
                         "of the multi-rank path; RCCL needs one GPU per rank)")
    ap.add_argument("--allreduce-dtype", choices=["bf16", "fp32"], default=None)
    ap.add_argument("--attention", choices=["slice", "sdpa", "flash"], default=None,
                    help="slice = the reference's stub (models.py:162-167, default); sdpa = "
                         "torch causal attention; flash = our causal flash kernel")
    ap.add_argument("--kernels", choices=["hip", "torch"], default=None)
    ap.add_argument("--model-size", default=None, help="override with a MODEL_CONFIGS size")
    ap.add_argument("--num-layers", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--output-dir", default=None)
    ap.add_argument("--graph", action="store_true",
                    help="(default where capturable) capture the forward in a HIP graph and "
                         "replay it: world 1, or all-reduces not issued through "
                         "ProcessGroupNCCL (custom / native / auto)")
    ap.add_argument("--eager", action="store_true",
                    help="time the forward issued eagerly from the host every iteration (the "
                         "reference's host-timed semantics, run_mpi.py:173-188) instead of "
                         "replaying the captured HIP graph")
    ap.add_argument("--trace", action="store_true",
                    help="emit roctx ranges (record with rocprofv3 --marker-trace)")
    ap.add_argument("--torch-profile", default=None, metavar="DIR",
                    help="torch.profiler Chrome trace per rank into DIR")
    ap.add_argument("--ignore-world-size", action="store_true",
                    help="accept any world size (reference exits on mismatch, run_mpi.py:73-77)")
    ap.add_argument("--shard-as", type=int, default=None, metavar="P",
                    help="world 1 only: run rank 0's shard of a P-way TP model (the exact "
                         "per-rank GEMM / LN shapes) with each all-reduce replaced by a local "
                         "stand-in (one rank's one-shot HBM traffic; + link time with "
                         "--emulate-busbw); output <backend>_<name>_shard<P>.json")
    ap.add_argument("--emulate-busbw", type=float, default=None, metavar="GBPS",
                    help="with --shard-as: also hold 32 workgroups for the ring all-reduce time "
                         "bytes*2(P-1)/P / busBW per all-reduce")
    ap.add_argument("--overlap-chunks", type=int, default=None, metavar="N",
                    help="split the batch into N micro-batches and interleave them so each "
                         "row-parallel all-reduce (side comm stream) runs under the next "
                         "micro-batch's GEMMs (execution.overlap_chunks; 1 = blocking, as the "
                         "reference)")
    ap.add_argument("--chunk-streams", action="store_true",
                    help="with --overlap-chunks: each micro-batch on a compute stream of its own "
                         "(verified concurrent, parallel/streams.py)")
    ap.add_argument("--check-dense", action="store_true",
                    help="after warmup, load the TP shards from a dense world-1 model of the "
                         "same seed (built on every rank) and report the max error of the TP "
                         "output against it (needs world > 1 on real ranks)")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    # config + thread env BEFORE importing torch (reference sets it after: SURVEY §2.8 item 8)
    from ..utils.config import load_config, setup_environment

    config = load_config(args.config)
    setup_environment(config)

    import numpy as np
    import torch

    from ..data import create_dataset_from_config
    from ..models.tp_transformer import MODEL_CONFIGS, create_model_from_config
    from ..parallel.comm import init_distributed
    from ..utils.io import save_results
    from ..utils.metrics import MetricsCollector, print_summary, rank_statistics
    from ..utils.sysinfo import collect_system_info

    ex = config["execution"]
    if args.allreduce:
        ex["allreduce"] = args.allreduce
    if args.allreduce_dtype:
        ex["allreduce_dtype"] = args.allreduce_dtype
    if args.attention:
        ex["attention"] = args.attention
    if args.kernels:
        ex["kernels"] = args.kernels
    if args.overlap_chunks:
        ex["overlap_chunks"] = args.overlap_chunks
    if args.model_size:
        config["model"].update(MODEL_CONFIGS[args.model_size])
        config["model"]["size"] = args.model_size
    if args.num_layers:
        config["model"]["num_layers"] = args.num_layers
    if args.warmup is not None:
        ex["warmup_iterations"] = args.warmup
    if args.iters is not None:
        ex["benchmark_iterations"] = args.iters
    if args.output_dir:
        config["experiment"]["output_dir"] = args.output_dir

    t0 = time.perf_counter()
    cpr = config["parallelism"].get("cores_per_rank")
    # host threads bound to the GPU's NUMA-local cores, cores_per_rank each (reference
    # launch_openmpi.sh:19-23 --bind-to core --map-by socket:PE=14)
    comm = init_distributed(args.backend,
                            device=None if args.device == "auto" else args.device,
                            cores_per_rank=int(cpr) if cpr else None)
    comm.install_tune_agreement()       # GEMM kernel choices agreed on rank-max timings
    comm.barrier()
    init_elapsed = time.perf_counter() - t0
    rank, world = comm.rank, comm.world_size

    expected = config["parallelism"]["world_size"]
    eff_world = args.shard_as or world
    if expected != "auto" and int(expected) != eff_world and not args.ignore_world_size:
        if rank == 0:
            print(f"ERROR: World size mismatch. Expected {expected}, got {eff_world}")
        comm.destroy()
        return 1
    model_comm = comm
    if args.shard_as:
        if world != 1 or args.shard_as < 2:
            if rank == 0:
                print("ERROR: --shard-as P needs world 1 and P >= 2")
            comm.destroy()
            return 1
        from ..parallel.comm import Comm

        # the model sees a P-rank world (shapes, per-rank FLOPs); no process group behind it
        model_comm = Comm(rank=0, world_size=args.shard_as, local_rank=comm.local_rank,
                          backend="emulate", device=comm.device)
        ex["allreduce"] = "emulate"

    if rank == 0:
        si = collect_system_info()
        print(f"\n{'=' * 60}\nExperiment: {config['experiment']['name']}\n"
              f"Backend: {args.backend.upper()} ({comm.backend})\n{'=' * 60}")
        print(f"World size: {world}\nInitialization time: {init_elapsed:.4f}s")
        print(f"Device: {si.get('gpu_name', 'cpu')} arch={si.get('gpu_arch')} "
              f"HIP={si.get('hip_version')} RCCL={si.get('rccl_version')}")
        m = config["model"]
        print(f"Model: {m.get('size')} H={m['hidden_size']} L={m['num_layers']} "
              f"heads={m['num_heads']} F={m['ffn_intermediate']}")
        print(f"Input: B={config['input']['batch_size']} S={config['input']['sequence_length']}")
        print(f"Execution: {ex}")

    model = create_model_from_config(config, model_comm)
    model.chunk_streams = bool(args.chunk_streams)
    if args.shard_as and args.emulate_busbw:
        from ..parallel.tensor_parallel import RowParallelLinear

        for m in model.modules():
            if isinstance(m, RowParallelLinear):
                m.emulate_busbw = float(args.emulate_busbw)
    dataset = create_dataset_from_config(config, comm.device)
    if rank == 0:
        print(f"[Rank 0] Model created: total params {model.get_num_parameters() / 1e9:.2f}B "
              f"(reference formula), {model.num_parameters_exact() / 1e9:.2f}B exact; "
              f"{model.get_memory_footprint() / 1e9:.2f} GB per rank")
    comm.barrier()

    metrics = MetricsCollector(rank, world)
    metrics.record_init_time(init_elapsed)
    gpu = comm.is_gpu

    fwd_bytes = 0
    for _ in range(int(ex["warmup_iterations"])):
        batch = dataset.get_batch()
        b0 = model.comm_bytes()
        t = time.perf_counter()
        model(batch)
        comm.sync()
        metrics.record_warmup_time(time.perf_counter() - t)
        fwd_bytes = model.comm_bytes() - b0
    comm.barrier()

    dense_check = None
    if args.check_dense and not args.shard_as:
        dense_check = _check_against_dense(config, comm, model, dataset.get_batch())
        if rank == 0:
            print(f"dense check: {dense_check}")

    run_forward = lambda: model(dataset.get_batch())  # noqa: E731
    # the timed loop replays a captured HIP graph wherever the forward is
    # capturable — the host issue cost of ~10 launches per layer (which made the eager TP
    # forward host-bound and GEMM tuning depend on the caller) is gone; --eager keeps the
    # reference's host-timed semantics
    use_graph = (not args.eager) and bool(ex.get("graph", True)) and gpu
    graph_note = None
    if use_graph and world > 1:
        # a layer whose all-reduce would go through ProcessGroup all_reduce (e.g.
        # allreduce=auto when the native engine could not be created on some rank) cannot be
        # captured; the decision is agreed, so every rank takes the same path
        if not all(comm.all_gather_object(_all_reduces_capturable(model))):
            graph_note = ("an all-reduce path is not capturable on some rank (no native engine "
                          "/ custom kernel)")
            use_graph = False
    if use_graph:
        # HIP graph: one replay launches the whole forward (all GEMM / LN / all-reduce kernels);
        # the autotuned GEMM choices were fixed by the eager warmup above. Any capture failure
        # on any rank -> every rank runs eagerly (agreed over the host side channel BEFORE the
        # first replay, so no rank replays collectives its peers never enqueue)
        static_in = dataset.get_batch()
        graph, err = None, None
        try:
            side = torch.cuda.Stream(comm.device)
            side.wait_stream(torch.cuda.current_stream(comm.device))
            with torch.cuda.stream(side):
                model(static_in)
            torch.cuda.current_stream(comm.device).wait_stream(side)
            comm.sync()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                model(static_in)
        except Exception as e:  # noqa: BLE001 - agreed below, then eager
            err = f"{type(e).__name__}: {e}"[:500]
            graph = None
        torch.cuda.synchronize(comm.device)
        errs = _agree_host(comm, err)
        if errs:
            graph_note = f"capture failed on rank(s) {sorted(errs)}: {errs[min(errs)]}"
            use_graph = False
        else:
            graph.replay()
            comm.sync()
            run_forward = graph.replay
    if graph_note and rank == 0:
        print(f"note: HIP graph replay off, running eagerly: {graph_note}")

    from ..utils import tracing

    if args.trace:
        tracing.enable()
    prof = tracing.torch_profile(args.torch_profile, rank)
    prof.__enter__()
    ev = []
    for _ in range(int(ex["benchmark_iterations"])):
        comm.barrier()                          # reference run_mpi.py:177
        if gpu:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
        t = time.perf_counter()
        with tracing.range("tp_forward"):
            run_forward()
        if gpu:
            e.record()
        comm.sync()
        comm.barrier()                          # reference run_mpi.py:183
        metrics.record_forward_time(time.perf_counter() - t)
        if gpu:
            ev.append(s.elapsed_time(e) * 1e-3)
    prof.__exit__(None, None, None)
    car = getattr(model, "ipc_allreduce", lambda: None)()
    if car is not None:                 # a timed-out IPC all-reduce must not pass silently
        car.raise_if_error()
    calibration = car.calibration if car is not None else None
    ar_bytes = fwd_bytes
    if ev:
        metrics.metrics["forward_device_times"] = ev

    summary = metrics.get_summary()
    # next to forward_mean: the reference host-times EAGER forwards
    # (run_mpi.py:173-185); a graph-replayed forward is not the same quantity
    summary["timing_mode"] = "hip_graph_replay" if use_graph else "eager"
    means = comm.all_gather_object(summary["forward_mean"])
    affinity = comm.affinity_all_ranks()
    if rank == 0:
        rs = rank_statistics(means)
        B, S = int(config["input"]["batch_size"]), int(config["input"]["sequence_length"])
        fwd = summary["forward_mean"]
        extra = {
            "tokens_per_s": B * S / fwd,
            "tflops_per_rank": model.flops_per_forward(B, S) / fwd / 1e12,
            "allreduce_bytes_per_forward_per_rank": ar_bytes,
            "allreduces_per_forward": 2 * int(config["model"]["num_layers"]),
            "forward_device_mean": float(np.mean(ev)) if ev else None,
            "kernels": ex.get("kernels"),
            "hip_graph": use_graph,
            "hip_graph_note": graph_note,
            "timing_mode": "hip_graph_replay" if use_graph else "eager",
            "gemm_tune_timing": __import__(
                "distributed_llm_backend_benchmark_amd.ops.gemm", fromlist=["x"]).tune_timing(),
            "gemm_fallbacks": __import__(
                "distributed_llm_backend_benchmark_amd.ops.gemm", fromlist=["x"]).FALLBACKS["count"],
            "gemm_kernel_mix": __import__(
                "distributed_llm_backend_benchmark_amd.ops.gemm", fromlist=["x"]).kernel_mix(),
            # node-measured IPC-vs-RCCL crossovers behind allreduce=auto (None: RCCL only)
            "allreduce_calibration": calibration,
            "dense_check": dense_check,
            # micro-batches interleaved so all-reduces run under GEMMs (1 = blocking)
            "overlap_chunks": model.overlap_split(
                torch.empty(B, 1, device="meta")),
            "chunk_streams": bool(args.chunk_streams),
        }
        if args.shard_as:
            extra["shard_as"] = {
                "P": args.shard_as, "emulate_busbw_GBps": args.emulate_busbw,
                "what": ("rank 0's shard of a P-way TP forward on ONE GPU: the exact per-rank "
                         "GEMM / LayerNorm shapes; each all-reduce replaced by a stand-in with "
                         "one rank's one-shot HBM traffic" +
                         (" plus the ring time at the assumed bus bandwidth"
                          if args.emulate_busbw else " (no link time)") +
                         "; tokens_per_s is the P-GPU job's (every rank holds all tokens)")}
        results = {
            "experiment": config["experiment"]["name"],
            "backend": args.backend,
            "config": config,
            "system_info": dict(collect_system_info(), host_affinity_per_rank=affinity),
            "rank_0_summary": summary,
            "rank_statistics": rs,
            "raw_metrics_rank_0": metrics.get_raw_metrics(),
            "throughput": extra,
        }
        print_summary(summary, args.backend.upper(), rank)
        print(f"\nRank Statistics:\n  Variance across ranks: {rs['variance_across_ranks']:.6g}"
              f"\n  Coefficient of variation: {rs['coefficient_of_variation']:.4f}"
              f"\n  tokens/s: {extra['tokens_per_s']:.1f}  TFLOP/s/rank: "
              f"{extra['tflops_per_rank']:.1f}")
        suffix = f"_shard{args.shard_as}" if args.shard_as else ""
        if extra["overlap_chunks"] > 1:
            suffix += f"_ov{extra['overlap_chunks']}" + ("cs" if args.chunk_streams else "")
        out = os.path.join(config["experiment"]["output_dir"],
                           f"{args.backend}_{config['experiment']['name']}{suffix}.json")
        save_results(results, out, rank)
    comm.barrier()
    comm.destroy()
    return 0


def _all_reduces_capturable(model) -> bool:
    """Every row-parallel layer's all-reduce can be captured in a HIP graph: our native RCCL
    engine exists on the layer, or it is forced to the IPC kernel (``allreduce=custom``);
    ``emulate`` is local work. Otherwise ``RowParallelLinear._all_reduce`` may fall through to
    ProcessGroup ``all_reduce``."""
    from ..parallel.tensor_parallel import RowParallelLinear

    for m in model.modules():
        if isinstance(m, RowParallelLinear):
            if m.allreduce == "emulate":
                continue
            if m._native is None and not (m.allreduce == "custom" and m._car is not None):
                return False
    return True


def _agree_host(comm, err):
    """Every rank's error string (None = ok), gathered over the host side channel (a failed
    capture may leave the device communicator unusable); returns {rank: error} of the failed."""
    import torch.distributed as dist

    if comm.world_size == 1:
        return {0: err} if err else {}
    out = [None] * comm.world_size
    dist.all_gather_object(out, err, group=comm.cpu_group())
    return {r: e for r, e in enumerate(out) if e}


def _check_against_dense(config, comm, model, batch) -> dict:
    """Build the dense (world-1) model of the same seed on every rank, shard its weights into
    the TP model (``LLM.load_from_dense``), run both on ``batch`` and compare: the TP forward,
    all-reduces included, must reproduce the dense output to bf16 accuracy (the test of
    ``run_mpi.py``'s model the reference never runs, models.py:95)."""
    import torch

    from ..models.tp_transformer import create_model_from_config
    from ..parallel.comm import Comm

    solo = Comm(rank=0, world_size=1, local_rank=comm.local_rank, backend=comm.backend,
                device=comm.device)
    dense = create_model_from_config(config, solo)
    with torch.no_grad():
        y_ref = dense(batch).float()
        model.load_from_dense(dense.state_dict())
        del dense
        y = model(batch).float()
    comm.sync()
    scale = float(y_ref.abs().max())
    err = float((y - y_ref).abs().max())
    errs = comm.all_gather_object(err)
    rel = max(errs) / max(scale, 1e-30)
    return {"max_abs_err": max(errs), "ref_max_abs": scale, "rel_err": rel,
            "passed": bool(rel < 5e-2 and all(e == e for e in errs))}


if __name__ == "__main__":
    sys.exit(main())
