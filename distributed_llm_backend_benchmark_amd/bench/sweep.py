"""1D and 3D collective sweeps.

1D (reference ``collectives/1d/openmpi.py:204-300``, ``1d/dsccl.py:165-265``): for each op ×
size, rank-seeded data, W warmup + N timed iterations, per-rank timings gathered to rank 0,
one JSON per (op, size).

3D (reference ``collectives/3d/openmpi.py:125-236``, ``3d/dsccl.py:120-241``): op × batch ×
seq × hidden grid of bf16 ``[B, S, H]`` tensors. ``wire_dtype="fp32"`` reproduces the
reference MPI path that up-cast to fp32 before the collective (``3d/openmpi.py:43``), with the
cast done on-device by the HIP cast kernel instead of a host numpy round trip.

Differences by design: per-config failures write ``<stem>.error.json`` instead of being
silently skipped (reference ``1d/openmpi.py:254-267``); ``resume=True`` skips configs whose
result exists; results can be validated against closed forms.
"""

from __future__ import annotations

import os
import traceback
from typing import Dict, Iterable, List, Optional, Sequence

import torch

from ..parallel.collectives import DTYPES, DTYPE_NAMES, make_data, make_op
from ..parallel.comm import Comm
from ..utils import faults, tracing
from ..utils.io import save_json
from . import schema
from .timing import time_batched, time_per_iteration


def _agree(comm: Comm, exc: Optional[BaseException]) -> None:
    """All ranks agree that setup succeeded everywhere (avoid one rank entering a collective
    alone and hanging until the PG timeout); on failure EVERY rank raises with the failing
    ranks' errors, so rank 0's error record names the real cause."""
    errs = comm.all_gather_object(None if exc is None else f"{type(exc).__name__}: {exc}")
    bad = {r: e for r, e in enumerate(errs) if e is not None}
    if bad:
        raise RuntimeError(f"setup failed on rank(s) {sorted(bad)}: {bad}")


class WrongResult(RuntimeError):
    """The collective's output failed its closed-form check on some rank: the config is
    recorded as ``<stem>.error.json`` with ``invalid: "wrong_result"`` and never timed or turned
    into a statistic."""


def _validate(comm: Comm, op, shape, dtype, seed, label=("", ""), src_dtype=None) -> bool:
    # src_dtype: the dtype the data was generated in before a wire cast (3D sweep with
    # wire_dtype): the closed form must see the same rounded values the collective moves
    inputs = [make_data(shape, src_dtype or dtype, r, comm.device, seed).to(dtype)
              for r in range(comm.world_size)]
    op.reset()
    comm.sync()
    comm.barrier()
    op.run()
    comm.sync()
    if faults.maybe_corrupt(label[0], label[1], comm.rank, op.result()):
        comm.sync()
    rtol = 5e-2 if dtype in (torch.bfloat16, torch.float16) else 1e-4
    atol = 0.25 * comm.world_size if dtype in (torch.bfloat16, torch.float16) else 1e-4
    ok = op.check(inputs, rtol=rtol, atol=atol)
    return all(comm.all_gather_object(ok))


def _bench_one(comm: Comm, op_name: str, data: torch.Tensor, warmup: int, iters: int,
               timing: str, batched: bool, graph: bool, validate: bool, seed: int,
               op_opts: Dict, label: str = "", src_dtype=None) -> Dict:
    op = make_op(op_name, comm, data, **op_opts)
    out: Dict = {"op_impl": getattr(op, "impl", None) or comm.backend_label}
    if op_opts.get("out_of_place"):
        out["out_of_place"] = True
    if colocated(comm.world_size):
        out["colocated"] = True
    if validate:
        out["validated"] = _validate(comm, op, tuple(data.shape), data.dtype, seed,
                                     (op_name, label), src_dtype)
        if not out["validated"]:          # agreed on every rank by _validate
            op.close()
            raise WrongResult(f"{op_name} {label}: output failed the closed-form check on at "
                              f"least one of {comm.world_size} rank(s)")
    tr = time_per_iteration(comm, op, iters, warmup, method=timing)
    all_t = comm.gather_floats(tr.timings)
    all_h = comm.gather_floats(tr.host_timings)
    out.update(timings=all_t, host_timings=all_h, timing_method=tr.timing_method,
               message_bytes=op.message_bytes, num_elements=op.num_elements)
    if batched:
        mean = time_batched(comm, op, iters, warmup, graph=graph)
        out["batched_mean_s"] = comm.allreduce_max(mean)
        from .timing import graph_safe

        out["batched_method"] = ("hip_graph" if (graph and comm.is_gpu and graph_safe(op))
                                 else "back_to_back")
    if op.ipc_kernel() is not None:     # a timed-out IPC kernel must not pass silently
        op.ipc_kernel().raise_if_error()
    op.close()          # collective: releases IPC registrations (direct / registered ops)
    del op
    return out


class BelowRoofline(RuntimeError):
    """A timing below the memory / xGMI roofline: the call enqueued no (or only part of its)
    work — never a measurement."""


def colocated(P: int) -> bool:
    """Ranks sharing one device (rehearsals on a one-GPU box): no xGMI link in the path."""
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    return P > 1 and 0 < ndev < int(os.environ.get("LOCAL_WORLD_SIZE", P))


def roofline_guard(op_name: str, r: Dict, P: int, coloc: bool = False) -> None:
    """Raise :class:`BelowRoofline` when the per-iteration p50 (all ranks' iterations pooled,
    the stats convention), the rank-max p50 or the batched mean of a result ``r`` (as returned
    by :func:`_bench_one`) beats the physical floor of ``stats.bandwidth.min_seconds``."""
    import numpy as np

    from ..stats.bandwidth import roofline_violation
    from ..stats.stats1d import rank_max_p50

    nbytes = r["message_bytes"]
    t = r.get("timings") or []
    flat = [x for row in t for x in row]
    checks = []
    if flat:
        checks += [("p50", float(np.median(flat))), ("rank_max_p50", rank_max_p50(t))]
    if r.get("batched_mean_s") is not None:
        checks.append(("batched_mean", float(r["batched_mean_s"])))
    for what, sec in checks:
        why = roofline_violation(op_name, nbytes, sec, P, coloc)
        if why:
            raise BelowRoofline(f"below_roofline ({what}): {why}")


def p1_opts(comm: Comm, op_name: str, op_opts: Dict) -> Dict:
    """At one rank an IN-PLACE collective enqueues nothing (RCCL returns at once): time the
    out-of-place form on our native engine instead — a real device copy of the message, as
    bench.py does — where the op has one; other ops keep their options (and the roofline guard
    refuses an empty call)."""
    if comm.world_size != 1 or not comm.is_gpu or op_opts.get("impl") == "custom":
        return op_opts
    if op_name in ("allreduce", "broadcast", "reduce"):
        return dict(op_opts, impl="native", out_of_place=True)
    return op_opts


def _write(comm: Comm, path: str, record: Dict) -> None:
    if comm.rank == 0:
        save_json(record, path)
        print(f"  Saved: {os.path.basename(path)}", flush=True)


def _write_error(comm: Comm, path: str, info: Dict, exc: BaseException) -> None:
    if comm.rank == 0:
        err = dict(info)
        err["error"] = f"{type(exc).__name__}: {exc}"
        if isinstance(exc, BelowRoofline):
            err["invalid"] = "below_roofline"
        elif isinstance(exc, WrongResult):
            err["invalid"] = "wrong_result"
            err["validated"] = False
        err["traceback"] = traceback.format_exc(limit=8)
        save_json(err, path[:-5] + ".error.json")
        print(f"  ERROR {os.path.basename(path)}: {err['error']}", flush=True)


def run_1d_sweep(comm: Comm, *, ops: Sequence[str], sizes: Dict[str, int], dtype: str = "bf16",
                 warmup: int = 10, iters: int = 100, output_dir: str = "results/1d/rccl",
                 impl_name: str = "rccl", timing: str = "auto", batched: bool = False,
                 graph: bool = False, validate: bool = False, resume: bool = False,
                 seed: int = 42, op_opts: Optional[Dict] = None,
                 extra: Optional[Dict] = None) -> List[str]:
    tdt = DTYPES[dtype]
    dname = DTYPE_NAMES[tdt]
    written: List[str] = []
    if comm.rank == 0:
        os.makedirs(output_dir, exist_ok=True)
        print(f"1D sweep impl={impl_name} backend={comm.backend_label} world={comm.world_size} "
              f"dtype={dname} ops={list(ops)} sizes={list(sizes)} warmup={warmup} iters={iters}",
              flush=True)
    for op_name in ops:
        for size_name, n in sizes.items():
            path = os.path.join(output_dir, schema.filename_1d(impl_name, op_name,
                                                               comm.world_size, size_name))
            if resume and comm.broadcast_object(os.path.exists(path)):
                continue
            info = {"implementation": impl_name, "operation": op_name,
                    "num_ranks": comm.world_size, "data_size_name": size_name,
                    "num_elements": n, "dtype": dname}
            try:
                setup_exc = None
                try:
                    faults.maybe_fail("setup", op_name, size_name, comm.rank)
                    data = make_data((n,), tdt, comm.rank, comm.device, seed)
                except Exception as e:  # OOM etc.
                    setup_exc = e
                _agree(comm, setup_exc)
                faults.maybe_fail("run", op_name, size_name, comm.rank)
                with tracing.range(f"{impl_name}/{op_name}/{size_name}"):
                    r = _bench_one(comm, op_name, data, warmup, iters, timing, batched, graph,
                                   validate, seed, p1_opts(comm, op_name, op_opts or {}),
                                   size_name)
                roofline_guard(op_name, r, comm.world_size, colocated(comm.world_size))
                rec = schema.result_1d(
                    impl=impl_name, backend=comm.backend_label, op=op_name,
                    ranks=comm.world_size, size_name=size_name, num_elements=r["num_elements"],
                    dtype=dname, nbytes=r["message_bytes"], warmup=warmup, iters=iters,
                    timing_method=r["timing_method"], timings=r["timings"],
                    host_timings=r["host_timings"], batched_mean_s=r.get("batched_mean_s"),
                    extra={k: v for k, v in r.items() if k in ("validated", "op_impl",
                                                                  "batched_method",
                                                                  "out_of_place", "colocated")}
                    | dict(extra or {}))
                _write(comm, path, rec)
                written.append(path)
                del data
            except Exception as e:
                _write_error(comm, path, info, e)
                if comm.is_gpu:
                    torch.cuda.empty_cache()
    return written


def run_3d_sweep(comm: Comm, *, ops: Sequence[str], batch_sizes: Iterable[int],
                 seq_lengths: Iterable[int], hidden_dims: Iterable[int], dtype: str = "bf16",
                 wire_dtype: Optional[str] = None, warmup: int = 10, iters: int = 100,
                 output_dir: str = "results/3d/rccl", impl_name: str = "rccl",
                 timing: str = "auto", batched: bool = False, graph: bool = False,
                 validate: bool = False, resume: bool = False, seed: int = 42,
                 op_opts: Optional[Dict] = None, extra: Optional[Dict] = None) -> List[str]:
    tdt = DTYPES[dtype]
    wdt = DTYPES[wire_dtype] if wire_dtype else tdt
    written: List[str] = []
    if comm.rank == 0:
        os.makedirs(output_dir, exist_ok=True)
        print(f"3D sweep impl={impl_name} world={comm.world_size} dtype={DTYPE_NAMES[tdt]} "
              f"wire={DTYPE_NAMES[wdt]} ops={list(ops)}", flush=True)
    for op_name in ops:
        for b in batch_sizes:
            for s in seq_lengths:
                for h in hidden_dims:
                    path = os.path.join(output_dir, schema.filename_3d(
                        impl_name, op_name, comm.world_size, b, s, h))
                    if resume and comm.broadcast_object(os.path.exists(path)):
                        continue
                    info = {"implementation": impl_name, "operation": op_name,
                            "num_ranks": comm.world_size,
                            "tensor_shape": {"batch": b, "seq_len": s, "hidden_dim": h}}
                    try:
                        setup_exc = None
                        shape_name = f"b{b}_s{s}_h{h}"
                        try:
                            faults.maybe_fail("setup", op_name, shape_name, comm.rank)
                            data = make_data((b, s, h), tdt, comm.rank, comm.device, seed)
                            if wdt != tdt:
                                from ..ops import cast as ops_cast
                                data = ops_cast(data, wdt)
                        except Exception as e:
                            setup_exc = e
                        _agree(comm, setup_exc)
                        faults.maybe_fail("run", op_name, shape_name, comm.rank)
                        with tracing.range(f"{impl_name}/{op_name}/{shape_name}"):
                            r = _bench_one(comm, op_name, data, warmup, iters, timing, batched,
                                           graph, validate, seed,
                                           p1_opts(comm, op_name, op_opts or {}), shape_name,
                                           src_dtype=tdt)
                        roofline_guard(op_name, r, comm.world_size, colocated(comm.world_size))
                        rec = schema.result_3d(
                            impl=impl_name, backend=comm.backend_label, op=op_name,
                            ranks=comm.world_size, batch=b, seq_len=s, hidden_dim=h,
                            dtype=DTYPE_NAMES[tdt], wire_dtype=DTYPE_NAMES[wdt],
                            wire_bytes=r["message_bytes"], warmup=warmup, iters=iters,
                            timing_method=r["timing_method"], timings=r["timings"],
                            host_timings=r["host_timings"],
                            batched_mean_s=r.get("batched_mean_s"),
                            extra={k: v for k, v in r.items()
                                   if k in ("validated", "op_impl", "batched_method",
                                            "out_of_place", "colocated")}
                            | dict(extra or {}))
                        _write(comm, path, rec)
                        written.append(path)
                        del data
                    except Exception as e:
                        _write_error(comm, path, info, e)
                        if comm.is_gpu:
                            torch.cuda.empty_cache()
    return written
