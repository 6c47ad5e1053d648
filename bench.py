#!/usr/bin/env python3
"""Headline benchmark: all-reduce bus bandwidth on MI355X (RCCL over xGMI), one rank per GPU.

Metric (BASELINE.json): "all-reduce bus BW (GB/s) + p50 latency vs msg size at 1/2/4/8 MI355X".
Headline config: the reference's best 3D all-reduce data point — a bf16 activation tensor
``[8, 2048, 2048]`` (64 MiB per rank), reference busBW 5.46 GB/s at P=8
(``collectives/3d/stats/mpiccl/benchmark_statistics_3d_mpiccl_standard.csv:10``).

One "step" = one in-place SUM all-reduce of that tensor on every rank. W untimed warmup steps,
then EXACTLY K steps timed between [barrier + synchronize] and [synchronize]; the elapsed time is
the MAX over ranks. busBW follows nccl-tests: ``bytes / t * 2(P-1)/P`` — identically 0 at P=1
(no inter-GPU traffic), where ``vs_baseline`` is null (the reference has no P=1 data).
Per-GPU message size is fixed as N grows: weak scaling.

Side measurements (also in the JSON line): p50 latency of a 512 B all-reduce (reference best
22.9 µs at P=2, 32.0 µs at P=8) and busBW at 8 MiB (reference best 7.53 GB/s), the 1 KiB..1 GiB
all-reduce sweep, and ``baseline_configs``: BASELINE configs 3 (3D activation-shaped
all-gather + reduce-scatter grid), 4 (MoE uneven all-to-all) and 5 (GPT-2-small DDP step,
B16 x T1024 per GPU) as isolated, validated, roofline-guarded, time-boxed sections
(``bench/baseline_configs.py``) — a failing section records ``{"error": ...}`` and never costs
the headline.

Whole-run deadline (``--deadline-s``, default 420 s, rank-agreed): the headline all-reduce is
always measured and printed; every later part (remaining headline candidates, side runs, each
sweep size, each BASELINE config section) first checks the deadline and, once it has passed, is
recorded as ``skipped_deadline`` instead of run. ``wall_s`` in the JSON is the whole run.

Usage: ``python bench.py [--gpus N] [--steps K] [--warmup W]``; for N>1 launch with
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py``.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

# RCCL / HIP IPC on this pool support only the dmabuf path: set before torch initialises HIP
# (every launcher exports it too; the driver's scaling run starts bench.py directly)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

REF_BUSBW_GBPS = 5.46          # best 3D all-reduce busBW (P=8, 64 MiB bf16)
REF_LAT_512B_US = {2: 22.9, 8: 32.0}
REF_BUSBW_8MIB = 7.53


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--shape", default="8,2048,2048", help="B,S,H of the bf16 message")
    ap.add_argument("--impl", default="best", choices=["best", "rccl", "native", "custom"],
                    help="best = time RCCL through torch, RCCL through our native C++ engine and "
                         "the IPC xGMI kernel (if its self-test passed on every rank) during "
                         "warmup and run the fastest")
    ap.add_argument("--no-side", action="store_true", help="skip the 512 B / 8 MiB side runs")
    ap.add_argument("--no-sweep", action="store_true", help="skip the all-reduce size sweep")
    ap.add_argument("--sweep-max-mib", type=int, default=1024,
                    help="largest message of the all-reduce size sweep (MiB per rank)")
    # BASELINE configs 3-5 (bench/baseline_configs.py): side sections after the headline
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the BASELINE config 3/4/5 sections (3D AG+RS grid, MoE "
                         "all-to-all, GPT-2 DDP step)")
    ap.add_argument("--config-budget-s", type=float, default=60.0,
                    help="rank-agreed time box of each config section (checked between "
                         "configurations)")
    ap.add_argument("--grid", default=None, metavar="B,S,H;...",
                    help="config 3 shapes (default: bench.baseline_configs.GRID_3D)")
    ap.add_argument("--moe", default=None, metavar="TOKENS,HIDDEN;...",
                    help="config 4 payloads per rank (default: MOE_PAYLOADS)")
    ap.add_argument("--ddp-model", default=None,
                    metavar="LAYERS,HEADS,EMBD,VOCAB,BATCH,SEQ",
                    help="config 5 model (default: GPT-2 small, B16 x T1024 per GPU)")
    ap.add_argument("--ddp-steps", type=int, default=10)
    ap.add_argument("--deadline-s", type=float, default=420.0,
                    help="whole-run deadline (rank-agreed): parts after the headline are skipped "
                         "and recorded as skipped_deadline once it has passed")
    return ap.parse_args(argv)


class Deadline:
    """Rank-agreed whole-run deadline: every check is collective (max elapsed over ranks), so
    all ranks take the same skip decision at the same point and no rank is left alone in a
    collective."""

    def __init__(self, comm, seconds: float, t0: float):
        self.comm, self.seconds, self.t0 = comm, float(seconds), t0
        self.skipped = []

    def remaining(self) -> float:
        return self.seconds - self.comm.allreduce_max(time.perf_counter() - self.t0)

    def expired(self, what: str = "") -> bool:
        gone = self.remaining() <= 0
        if gone and what:
            self.skipped.append(what)
        return gone


def _shapes(spec):
    return [tuple(int(v) for v in part.split(",")) for part in spec.split(";") if part.strip()]


def _baseline_configs(comm, args, deadline=None) -> dict:
    """BASELINE configs 3/4/5 as isolated, validated, roofline-guarded, time-boxed sections
    (bench/baseline_configs.py): a failure is recorded as {"error": ...} for its section only;
    each section's time box is cut to what is left of the whole-run ``deadline`` and a section
    that starts after it is recorded as skipped."""
    from distributed_llm_backend_benchmark_amd.bench import baseline_configs as bc

    comm.cpu_group()        # host side channel for the sections' failure agreement (collective)
    gpu = comm.is_gpu
    # CPU (gloo plumbing) runs default to reduced shapes — the BASELINE shapes are GPU sizes
    grid = _shapes(args.grid) if args.grid else (bc.GRID_3D if gpu else [(1, 512, 1024)])
    moe = _shapes(args.moe) if args.moe else (bc.MOE_PAYLOADS if gpu else [(512, 1024)])
    model = None
    if not gpu and not args.ddp_model:
        model = dict(n_layer=2, n_head=2, n_embd=64, vocab=256, batch=2, seq=32)
    if args.ddp_model:
        keys = ("n_layer", "n_head", "n_embd", "vocab", "batch", "seq")
        model = dict(zip(keys, (int(v) for v in args.ddp_model.split(","))))
    sections = [
        ("config3_3d_allgather_reduce_scatter", "config3",
         lambda c, b: bc.grid_3d(c, b, shapes=grid)),
        ("config4_moe_alltoall", "config4", lambda c, b: bc.moe_alltoall(c, b, payloads=moe)),
        ("config5_gpt2_ddp", "config5",
         lambda c, b: bc.gpt2_ddp(c, b, steps=args.ddp_steps, model=model)),
    ]
    out = {}
    for key, name, fn in sections:
        budget = args.config_budget_s
        if deadline is not None:
            left = deadline.remaining()
            if left <= 0:
                deadline.skipped.append(key)
                out[key] = {"skipped_deadline": True}
                continue
            budget = min(budget, left)
        out[key] = bc.run_section(comm, name, fn, budget)
    return out


SWEEP_BYTES = [1 << 10, 8 << 10, 64 << 10, 512 << 10, 4 << 20, 32 << 20, 256 << 20, 1 << 30]


def _allreduce_sweep(comm, max_mib: int, deadline=None):
    """Mean time per call (back to back, rank max) of a bf16 SUM all-reduce per message size and
    implementation; per size the fastest VALIDATED one (one extra call on fresh data checked
    against an fp32 reference sum on every rank) is reported with busBW / algBW. Candidates: RCCL via
    torch, RCCL via our native engine, and (P > 1, self-test passed) the IPC xGMI kernel —
    staged one-/two-shot within its staging capacity, and in place on a registered buffer."""
    import torch
    import torch.distributed as dist

    from distributed_llm_backend_benchmark_amd.parallel.collectives import make_data, make_op
    from distributed_llm_backend_benchmark_amd.stats.bandwidth import algbw_gbps, busbw_gbps

    P = comm.world_size
    car = None
    if P > 1 and comm.is_gpu:
        from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import (
            get_custom_allreduce)

        car = get_custom_allreduce(comm)
    out = []
    for nbytes in SWEEP_BYTES:
        if nbytes > max_mib << 20:
            break
        if deadline is not None and deadline.expired(f"allreduce_sweep/{nbytes}"):
            out.append({"bytes": nbytes, "impl": None, "skipped_deadline": True})
            continue
        data = make_data((nbytes // 2,), torch.bfloat16, comm.rank, comm.device)
        flat = data.reshape(-1)
        if P == 1 and comm.is_gpu:
            # one rank: an in-place all-reduce enqueues no GPU work; time the out-of-place form
            # (the identity all-reduce = a real device copy of the message)
            cands = [("native_oop", {"impl": "native", "out_of_place": True})]
        else:
            cands = [("rccl", {"impl": "rccl"})]
            if comm.is_gpu:
                cands.append(("native", {"impl": "native"}))
        if car is not None and car.healthy and car.supports(flat):
            cands.append(("custom", {"impl": "custom"}))
        if car is not None and car.reg_healthy and car.supports_registered(flat):
            cands.append(("custom_reg", {"impl": "custom_reg", "nblocks": 256}))
        iters = 50 if nbytes <= 4 << 20 else 20 if nbytes <= 32 << 20 else 8
        ref = data.float()                  # fp32 reference sum through the process group
        if P > 1:
            dist.all_reduce(ref)
        res, invalid = {}, []
        for label, opts in cands:
            try:
                op = make_op("allreduce", comm, data, **opts)
            except RuntimeError:            # agreed on every rank (collective health flags)
                continue
            for _ in range(3):
                op.run()
            comm.sync()
            t = _timed_steps(comm, op, iters) / iters
            if _checked(comm, op, ref):
                res[label] = t
            else:
                invalid.append(label)
            op.close()                      # releases its IPC registration (collective)
            del op
        if not res:
            out.append({"bytes": nbytes, "impl": None, "invalid": invalid})
            continue
        for k in [k for k, v in res.items() if too_fast("allreduce", nbytes, v, P)]:
            invalid.append(f"{k}:below_roofline")   # an empty call, not a measurement
            del res[k]
        if not res:
            out.append({"bytes": nbytes, "impl": None, "invalid": invalid})
            continue
        best = min(res, key=res.get)
        t = res[best]
        out.append({"bytes": nbytes, "impl": best, "us": round(t * 1e6, 2),
                    "busbw_GBps": float(f"{busbw_gbps('allreduce', nbytes, t, P):.4g}"),
                    "algbw_GBps": float(f"{algbw_gbps('allreduce', nbytes, t, P):.4g}"),
                    "us_by_impl": {k: round(v * 1e6, 2) for k, v in res.items()},
                    **({"invalid": invalid} if invalid else {})})
        del data, flat
    return out


def too_fast(op_name: str, nbytes: int, seconds: float, P: int):
    """The reason a timing is physically impossible (below the traffic-based memory / xGMI
    roofline of ``stats.bandwidth.min_seconds``: the call enqueued no work), else None."""
    import torch

    from distributed_llm_backend_benchmark_amd.stats.bandwidth import roofline_violation

    # ranks sharing one device (a rehearsal on a one-GPU box): no xGMI link in the path
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    colocated = P > 1 and 0 < ndev < int(os.environ.get("LOCAL_WORLD_SIZE", P))
    return roofline_violation(op_name, nbytes, seconds, P, colocated)


def _checked(comm, op, ref) -> bool:
    """One all-reduce on fresh data compared with the fp32 reference sum ``ref``; collective:
    True only if it matched on every rank (a candidate that fails is never reported)."""
    import torch

    op.reset()
    op.run()
    comm.sync()
    ok = bool(torch.allclose(op.result().float(), ref, rtol=2e-2,
                             atol=5e-2 * comm.world_size))
    return all(comm.all_gather_object(ok))


def _timed_steps(comm, op, steps: int) -> float:
    import torch  # noqa: F401

    comm.barrier()
    comm.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        op.run()
    comm.sync()
    dt = time.perf_counter() - t0
    return comm.allreduce_max(dt)


def main(argv=None) -> int:
    t_start = time.perf_counter()
    args = parse(argv)
    import torch

    from distributed_llm_backend_benchmark_amd.bench.timing import time_per_iteration
    from distributed_llm_backend_benchmark_amd.parallel.collectives import make_data, make_op
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.stats.bandwidth import algbw_gbps, busbw_gbps

    backend = "rccl" if torch.cuda.is_available() else "gloo"
    # DLBB_BENCH_BACKEND=gloo with GPUs visible: gloo process group over GPU tensors — lets
    # several ranks share one GPU to rehearse the multi-rank path (IPC kernel, candidate
    # agreement, native-engine refusal of duplicate GPUs); never used for reported numbers
    override = os.environ.get("DLBB_BENCH_BACKEND")
    if override:
        comm = init_distributed(override, timeout_s=900,
                                device="cuda" if torch.cuda.is_available() else None)
    else:
        comm = init_distributed(backend, timeout_s=900)
    P = comm.world_size
    deadline = Deadline(comm, args.deadline_s, t_start)
    if args.gpus != P and comm.rank == 0:
        print(f"note: --gpus {args.gpus} but world size is {P}; using {P}", file=sys.stderr)

    B, S, H = (int(x) for x in args.shape.split(","))
    data = make_data((B, S, H), torch.bfloat16, comm.rank, comm.device)
    # candidates: (label, impl, opts); every rank builds the same list (the custom kernel's
    # health flags are agreed collectively), so trial construction stays collective-safe
    cands = []
    if P == 1 and comm.is_gpu:
        # one rank: in-place all-reduces (RCCL or native) enqueue no GPU work, so the only
        # candidate is the out-of-place identity all-reduce, a real HBM copy of the message
        cands.append(("native_oop", "native", {"out_of_place": True}))
    else:
        if args.impl in ("best", "rccl"):
            cands.append(("rccl", "rccl", {}))
        if args.impl in ("best", "native") and comm.is_gpu:
            cands.append(("native", "native", {}))
    if args.impl in ("best", "custom") and P > 1 and comm.is_gpu:
        from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import (
            get_custom_allreduce)

        car = get_custom_allreduce(comm)
        flat = data.reshape(-1)
        if car is not None and car.healthy and car.supports(flat):
            cands += [("custom", "custom", {}), ("custom/nb256", "custom", {"nblocks": 256})]
        if car is not None and car.reg_healthy and car.supports_registered(flat):
            # in place on an IPC-registered buffer: no copy-in / staging pass
            cands += [(f"custom_reg/nb{nb}", "custom_reg", {"nblocks": nb})
                      for nb in (64, 128, 256)]
            if car.push_healthy and flat.numel() * flat.element_size() <= car.capacity:
                # same traffic as posted remote writes (peer staging + result pushes)
                cands += [(f"custom_push/nb{nb}", "custom_reg", {"nblocks": nb, "push": True})
                          for nb in (128, 256)]
        if args.impl == "custom" and not cands:
            raise SystemExit("custom all-reduce unavailable (setup or self-test failed)")
    calibration = None
    if P > 1 and comm.is_gpu and args.impl in ("best", "custom"):
        # the node-measured IPC-vs-RCCL crossovers the library's "auto" policy uses (rank-max,
        # agreed on every rank; parallel/custom_allreduce.py calibrate)
        calibration = getattr(car, "calibration", None) if car is not None else None
    trial, invalid = {}, []
    op, op_label = None, None
    ref = data.float()                  # fp32 reference sum: every candidate is checked once
    if P > 1:
        import torch.distributed as dist

        dist.all_reduce(ref)
    for label, impl, opts in cands:
        if op is not None and deadline.expired(f"headline_candidate/{label}"):
            continue                        # keep the best candidate timed so far
        try:
            cand = make_op("allreduce", comm, data, impl=impl, **opts)
        except RuntimeError as e:      # e.g. native engine init failed (agreed on all ranks)
            if args.impl != "best":
                raise
            if comm.rank == 0:
                print(f"note: {label} all-reduce unavailable: {e}", file=sys.stderr)
            continue
        if not _checked(comm, cand, ref):
            invalid.append(label)
            if comm.rank == 0:
                print(f"note: {label} all-reduce gave a wrong sum; not used", file=sys.stderr)
            cand.close()
            continue
        for _ in range(max(1, args.warmup)):
            cand.run()
        comm.sync()
        trial[label] = _timed_steps(comm, cand, 10) / 10 if len(cands) > 1 else 0.0
        if op is None or trial[label] < trial[op_label]:
            if op is not None:
                op.close()                  # trial times are rank-max: same choice everywhere
            op, op_label = cand, label
        else:
            cand.close()
    if op is None:
        raise SystemExit(f"no all-reduce implementation passed its check: {invalid}")
    nbytes = op.message_bytes
    for _ in range(args.warmup):
        op.run()
    comm.sync()
    total = _timed_steps(comm, op, args.steps)
    per_step = total / args.steps
    if op.ipc_kernel() is not None:     # collective: raise everywhere after an IPC timeout
        op.ipc_kernel().raise_if_error()
    bus = busbw_gbps("allreduce", nbytes, per_step, P)
    alg = algbw_gbps("allreduce", nbytes, per_step, P)
    why = too_fast("allreduce", nbytes, per_step, P)
    if why:
        raise SystemExit(f"{why}: {op_label} timed an empty call, refusing to report it")

    side = {}
    if not args.no_side and deadline.expired("side_512B_8MiB"):
        side = {"side_skipped_deadline": True}
    elif not args.no_side:
        small_opts = ({"impl": "native", "out_of_place": True} if P == 1 and comm.is_gpu
                      else {"impl": "auto"})
        # 512 B latency candidates: the size policy (IPC one-shot below the crossover, else RCCL)
        # and, at P > 1, the registered in-place two-shot (no copy-in; fastest form in the
        # single-GPU emulation, profiles/r02_car_harness); each validated before it is timed
        lat_cands = [("auto", small_opts)]
        if P > 1 and comm.is_gpu:
            from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import (
                get_custom_allreduce)

            car_s = get_custom_allreduce(comm)
            if car_s is not None and car_s.reg_healthy:
                lat_cands.append(("custom_reg", {"impl": "custom_reg", "nblocks": 1}))
        sdata = make_data((256,), torch.bfloat16, comm.rank, comm.device)
        sref = sdata.float()
        if P > 1:
            import torch.distributed as dist

            dist.all_reduce(sref)
        lat_samples, lat_invalid = {}, []
        for label, opts in lat_cands:
            try:
                small = make_op("allreduce", comm, sdata, **opts)
            except RuntimeError:            # agreed on every rank (collective health flags)
                continue
            if P > 1 and not _checked(comm, small, sref):
                lat_invalid.append(label)
                small.close()
                continue
            tr = time_per_iteration(comm, small, iters=100, warmup=10)
            lat_samples[getattr(small, "impl", label)] = comm.gather_floats(tr.timings)
            small.close()
        lat_native = None
        if comm.is_gpu:
            try:
                from distributed_llm_backend_benchmark_amd.parallel.rccl_native import get_native

                eng = get_native(comm)
                sb = make_data((256,), torch.bfloat16, comm.rank, comm.device)
                rb = torch.empty_like(sb) if P == 1 else sb   # one rank: out of place (a copy)
                # per-iteration loop in C++: device barrier, event, all-reduce, event
                lat_native = comm.gather_floats(eng.time_iters("allreduce", sb, rb, 256,
                                                               iters=100, warmup=10))
            except RuntimeError as e:
                if comm.rank == 0:
                    print(f"note: native 512 B timing unavailable: {e}", file=sys.stderr)
        mid = make_op("allreduce", comm, make_data((4 * 1024 * 1024,), torch.bfloat16,
                                                   comm.rank, comm.device),
                      **(small_opts if P == 1 else {"impl": op.impl}))
        for _ in range(5):
            mid.run()
        mid_t = _timed_steps(comm, mid, 20) / 20
        mid.close()
        if comm.rank == 0:
            import numpy as np

            # p50 over all ranks' iterations (reference stats pool [rank][iter])
            lats = {k: float(np.median(np.asarray(v, dtype=np.float64))) * 1e6
                    for k, v in lat_samples.items()}
            if lat_native is not None:
                lats["native"] = float(np.median(np.asarray(lat_native, dtype=np.float64))) * 1e6
            best = min(lats, key=lats.get) if lats else None
            side = {} if best is None else {
                "p50_latency_us_512B": lats[best],
                "p50_latency_512B_impl": best,
                "p50_latency_us_512B_by_impl": lats,
                **({"p50_latency_512B_invalid": lat_invalid} if lat_invalid else {}),
                "ref_p50_latency_us_512B": REF_LAT_512B_US.get(P),
                "busbw_GBps_8MiB": busbw_gbps("allreduce", 8 << 20, mid_t, P),
                "ref_busbw_GBps_8MiB": REF_BUSBW_8MIB,
            }

    # the BASELINE.json metric is busBW + latency *vs message size*: a 1 KiB .. 1 GiB all-reduce
    # sweep (bf16) in the same run, best implementation per size (every rank builds the same
    # candidate list; health flags are agreed collectively), so each N of the driver's scaling
    # runs carries the whole curve
    sweep = []
    if not args.no_side and not args.no_sweep:
        sweep = _allreduce_sweep(comm, args.sweep_max_mib, deadline)

    # BASELINE configs 3/4 on the same [B,S,H] message at P > 1: all-gather, reduce-scatter and
    # all-to-all through RCCL and through the direct one-hop IPC kernels (side measurements)
    coll = {}
    if not args.no_side and P > 1:
        for name in ("allgather", "reduce_scatter", "alltoall"):
            if deadline.expired(f"collectives_same_message/{name}"):
                coll[name] = {"skipped_deadline": True}
                continue
            res = {}
            for label, opts in (("rccl", {}), ("direct_ipc", {"direct": True})):
                if label == "direct_ipc" and not comm.is_gpu:
                    continue
                try:
                    cop = make_op(name, comm, data, **opts)
                except RuntimeError as e:   # agreed on every rank (health flags are collective)
                    if comm.rank == 0:
                        print(f"note: {name}/{label} unavailable: {e}", file=sys.stderr)
                    continue
                for _ in range(3):
                    cop.run()
                comm.sync()
                t = _timed_steps(comm, cop, 10) / 10
                why = too_fast(name, cop.message_bytes, t, P)
                res[label] = ({"invalid": why} if why else
                              {"busbw_GBps": busbw_gbps(name, cop.message_bytes, t, P),
                               "ms": t * 1e3})
                cop.close()
                del cop
            coll[name] = res

    # one GPU: the IPC collective kernels measured with W virtual ranks in this process
    # (parallel/virtual_ranks.py) — protocol latency and in-place two-shot time on one HBM,
    # validated against an fp32 sum first; NOT inter-GPU numbers (never used for "value")
    emulation = None
    if (P == 1 and comm.is_gpu and not args.no_side
            and deadline.expired("virtual_rank_emulation")):
        emulation = {"skipped_deadline": True}
    elif P == 1 and comm.is_gpu and not args.no_side:
        try:
            from distributed_llm_backend_benchmark_amd.parallel.virtual_ranks import (
                emulation_summary)

            emulation = emulation_summary(big_bytes=nbytes)
        except Exception as e:  # noqa: BLE001 - side measurement only
            emulation = {"error": repr(e)}

    # BASELINE configs 3-5 at this N (the driver's scaling run measures every config)
    configs = {}
    if not args.no_configs:
        configs = _baseline_configs(comm, args, deadline)
    affinity = comm.affinity_all_ranks() if comm.is_gpu else None   # collective
    wall = comm.allreduce_max(time.perf_counter() - t_start)

    if comm.rank == 0:
        rec = {
            "metric": "all-reduce bus BW (GB/s)",
            "value": round(bus, 4),
            "unit": "GB/s",
            "n_gpus": P,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(bus / REF_BUSBW_GBPS, 3) if P > 1 else None),
            "dtype": "bf16",
            "data": "synthetic (rank-seeded randn, on device)",
            "config": {
                "model": f"allreduce_3d_b{B}_s{S}_h{H}",
                "global_batch": B,
                "seq_len": S,
                "hidden": H,
                "message_bytes_per_rank": nbytes,
                "parallelism": f"{'rccl' if comm.backend == 'nccl' else comm.backend}_world{P}",
                "impl": op_label,
                "impl_trial_ms": {k: v * 1e3 for k, v in trial.items()} if len(trial) > 1 else None,
                "impl_invalid": invalid or None,
            },
            "algbw_GBps": alg,
            "baseline_busbw_GBps": REF_BUSBW_GBPS,
            "note": ("busBW = bytes/t*2(P-1)/P (nccl-tests); identically 0 at P=1, where "
                     "vs_baseline is null (reference has no single-rank data)" +
                     ("; P=1 step = out-of-place identity all-reduce (a device copy of the "
                      "message: real GPU work, algBW = copy throughput); in-place candidates "
                      "enqueue nothing at one rank and are excluded" if P == 1 else "")),
            **side,
            "wall_s": round(wall, 2),
            "deadline_s": args.deadline_s,
            "skipped_deadline": deadline.skipped,
        }
        if calibration:
            rec["allreduce_calibration"] = calibration
        if coll:
            rec["collectives_same_message"] = coll
        if sweep:
            rec["allreduce_sweep"] = sweep
        if configs:
            rec["baseline_configs"] = configs
        if affinity:
            rec["host_affinity_per_rank"] = affinity    # NUMA-local core binding per rank
        if emulation is not None:
            rec["virtual_rank_emulation"] = {
                "what": ("IPC all-reduce kernels, W ranks emulated on ONE GPU (one fused launch "
                         "of the production device code; all traffic through one HBM, not "
                         "xGMI): one-shot 512 B latency and registered two-shot on the headline "
                         "message, us per call back to back"),
                **emulation}
        print(json.dumps(rec), flush=True)
    comm.barrier()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
