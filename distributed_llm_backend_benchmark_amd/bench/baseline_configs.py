"""BASELINE configs 3-5 measured inside ``bench.py`` at N ranks.

The driver's only multi-GPU command is ``bench.py`` at 1/2/4/8 GPUs. Its headline is the
all-reduce (configs 1/2); this module adds the other three BASELINE.json configs as side
sections of the same run, so a scaling run on an 8-GPU node captures every config with no code
change:

* **config 3** — 3D activation-shaped all-gather + reduce-scatter on a grid of ``[B, S, H]``
  bf16 messages (reference grid ``collectives/3d/openmpi.py:19-31``; ops
  ``collectives/3d/openmpi.py:55-70`` / ``3d/dsccl.py:60-70``), through RCCL (torch process
  group), our native C++ RCCL engine and the direct one-hop IPC kernels (P > 1).
* **config 4** — MoE-shaped uneven all-to-all (expert-parallel dispatch; the reference only has
  the equal-split ``alltoall``, ``collectives/1d/openmpi.py:154-171``) at two token payloads,
  through RCCL, the native engine and our one-hop IPC all-to-all-v kernel.
* **config 5** — a GPT-2-small DDP training step, B16 x T1024 per GPU (the reference's only
  data-parallel step is ``test/ccl.py:92-115``), once per bucket all-reduce path
  (``auto`` / ``rccl`` / ``native`` / ``custom``), the fastest on rank-max ms/step reported.

Every section is
* **validated** — each candidate's result is compared with a closed form rebuilt from the
  rank-seeded inputs before it is reported (copies bit-exact, sums to bf16 tolerance);
* **roofline-guarded** — a time below the memory / xGMI floor (``stats.bandwidth``) is an empty
  call, recorded as ``invalid`` and never as a bandwidth;
* **time-boxed** — a rank-agreed budget is checked between configurations;
* **isolated** — an exception in a section becomes ``{"error": ...}`` for that section (agreed
  on every rank over the host side channel), never a lost headline line.
"""

from __future__ import annotations

import os
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..parallel.collectives import make_data, make_op
from ..parallel.comm import Comm
from ..stats.bandwidth import algbw_gbps, busbw_gbps, roofline_violation

# config 3: activation shapes [B, S, H] (bf16), VERDICT r03 item 1(a) — 64 MiB .. 512 MiB per rank
GRID_3D: List[Tuple[int, int, int]] = [(8, 2048, 4096), (16, 4096, 4096), (1, 8192, 4096),
                                       (32, 2048, 2048)]
GRID_3D_OPS = ("allgather", "reduce_scatter")
# config 4: (tokens per rank, hidden) of the MoE dispatch payload — 32 MiB and 128 MiB per rank
MOE_PAYLOADS: List[Tuple[int, int]] = [(4096, 4096), (16384, 4096)]
# config 5: GPT-2 small, micro-batch 16 x 1024 tokens per GPU
GPT2_SMALL = dict(n_layer=12, n_head=12, n_embd=768, vocab=50304, batch=16, seq=1024)


class SectionFailed(RuntimeError):
    pass


class Budget:
    """A rank-agreed time box: :meth:`exhausted` is collective (rank-max elapsed time), so every
    rank stops at the same configuration."""

    def __init__(self, comm: Comm, seconds: float):
        self.comm, self.seconds, self.t0 = comm, float(seconds), time.perf_counter()

    def elapsed(self) -> float:
        return time.perf_counter() - self.t0

    def exhausted(self) -> bool:
        return self.comm.allreduce_max(self.elapsed()) > self.seconds


def _agree_errors(comm: Comm, err: Optional[str]) -> Dict[int, str]:
    """Every rank's error string (None = ok) over the host side channel — usable after a
    device-side failure broke the RCCL communicator."""
    if comm.world_size == 1:
        return {0: err} if err else {}
    out: List[Optional[str]] = [None] * comm.world_size
    dist.all_gather_object(out, err, group=comm.cpu_group())
    return {r: e for r, e in enumerate(out) if e}


def local_step(comm: Comm, fn: Callable[[], object]):
    """Run rank-local work that can fail on one rank only (allocation, input generation), then
    agree over the side channel before anyone enters a collective: if it failed anywhere, EVERY
    rank raises (naming the failing ranks) instead of one rank leaving the others blocked in the
    next collective until the process-group timeout."""
    err, out = None, None
    try:
        out = fn()
    except Exception as e:  # noqa: BLE001 - agreed below
        err = f"{type(e).__name__}: {e}"[:1000]
    bad = _agree_errors(comm, err)
    if bad:
        raise SectionFailed(f"local step failed on rank(s) {sorted(bad)}: {bad[min(bad)]}")
    return out


def _inject(name: str, rank: int) -> None:
    inj = os.environ.get("DLBB_BENCH_FAIL_SECTION", "")
    if inj:
        sec, _, rk = inj.partition(":")
        if sec == name and (not rk or int(rk) == rank):
            raise SectionFailed(f"injected failure in section {name} on rank {rank}")


def run_section(comm: Comm, name: str, fn: Callable[[Comm, Budget], Dict],
                budget_s: float) -> Dict:
    """Run one section on every rank; an exception anywhere becomes ``{"error": ...}`` on every
    rank (agreed), so the caller's headline record is never lost. Fault injection for tests:
    ``DLBB_BENCH_FAIL_SECTION=<name>[:<rank>]`` fails that section's first local step."""
    t0 = time.perf_counter()
    err, res = None, None
    try:
        local_step(comm, lambda: _inject(name, comm.rank))
        res = fn(comm, Budget(comm, budget_s))
    except Exception as e:  # noqa: BLE001 - recorded, never fatal to the headline
        err = f"{type(e).__name__}: {e}"[:2000]
    bad = _agree_errors(comm, err)
    if comm.is_gpu:
        torch.cuda.empty_cache()
    if bad:
        first = min(bad)
        return {"error": bad[first], "failed_ranks": sorted(bad),
                "seconds": round(time.perf_counter() - t0, 2)}
    res = dict(res or {})
    res["seconds"] = round(comm.allreduce_max(time.perf_counter() - t0), 2)
    return res


# ------------------------------------------------------------------------------ helpers
def _colocated(P: int) -> bool:
    """Ranks sharing one device (rehearsals): no xGMI link in the path."""
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    return P > 1 and 0 < ndev < int(os.environ.get("LOCAL_WORLD_SIZE", P))


def _time_back_to_back(comm: Comm, op, iters: int, warmup: int = 3) -> float:
    """Mean seconds per call of ``iters`` back-to-back calls, [barrier + sync] .. [sync], rank
    max (nccl-tests methodology, as the headline)."""
    for _ in range(warmup):
        op.run()
    comm.sync()
    comm.barrier()
    comm.sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        op.run()
    comm.sync()
    return comm.allreduce_max(time.perf_counter() - t0) / iters


def _candidates(comm: Comm, direct: bool = True) -> List[Tuple[str, Dict]]:
    out = [("rccl", {})]
    if comm.is_gpu:
        out.append(("native", {"impl": "native"}))
        if direct and comm.world_size > 1:
            out.append(("direct_ipc", {"direct": True}))
    return out


def _inputs(comm: Comm, shape, r: int) -> torch.Tensor:
    return make_data(shape, torch.bfloat16, r, comm.device).reshape(-1)


def validate_result(comm: Comm, op_name: str, op, shape) -> bool:
    """Collective: ``op``'s result on fresh data equals the closed form rebuilt from every rank's
    seeded input (streamed one rank at a time, so a P x 512 MiB all-gather needs no P-fold
    fp32 copy). Copies (all-gather, all-to-all) must be bit-exact; sums within bf16 tolerance."""
    op.reset()
    comm.sync()
    comm.barrier()
    op.run()
    comm.sync()
    P, me = comm.world_size, comm.rank
    got = op.result()
    ok = True
    if op_name == "allgather":
        n = int(torch.Size(shape).numel())
        for r in range(P):
            ok &= bool(torch.equal(got[r * n:(r + 1) * n], _inputs(comm, shape, r)))
    elif op_name == "reduce_scatter":
        n = op.inp.numel() // P
        acc = torch.zeros(n, dtype=torch.float32, device=comm.device)
        for r in range(P):
            acc += _inputs(comm, shape, r)[me * n:(me + 1) * n].float()
        ok = bool(torch.allclose(got.float(), acc, rtol=2e-2, atol=5e-2 * P))
    elif op_name == "alltoall_moe":
        parts = []
        for r in range(P):
            off = sum(op.mat[r][:me])
            parts.append(_inputs(comm, shape, r)[off:off + op.mat[r][me]])
        ok = bool(torch.equal(got, torch.cat(parts)))
    else:
        raise ValueError(op_name)
    if comm.world_size == 1:
        return ok
    return all(comm.all_gather_object(ok))


def _measure(comm: Comm, op_name: str, shape, data: torch.Tensor, label: str, opts: Dict,
             iters: int) -> Dict:
    """One (op, message, implementation) cell: build, validate, time, guard. Construction
    failures are agreed on every rank by the op constructors (health flags are collective)."""
    try:
        op = make_op(op_name, comm, data, **opts)
    except (RuntimeError, KeyError) as e:
        return {"unavailable": str(e)[:300]}
    try:
        if not validate_result(comm, op_name, op, shape):
            return {"invalid": "wrong result"}
        t = _time_back_to_back(comm, op, iters)
        if op.ipc_kernel() is not None:         # collective: a timed-out IPC wait raises
            op.ipc_kernel().raise_if_error()
        nbytes = op.message_bytes
        why = roofline_violation(op_name, nbytes, t, comm.world_size, _colocated(comm.world_size))
        if why:
            return {"invalid": why}
        return {"ms": round(t * 1e3, 4),
                "busbw_GBps": float(f"{busbw_gbps(op_name, nbytes, t, comm.world_size):.4g}"),
                "algbw_GBps": float(f"{algbw_gbps(op_name, nbytes, t, comm.world_size):.4g}")}
    finally:
        op.close()                               # collective: releases IPC registrations


def _best(cells: Dict[str, Dict]) -> Optional[str]:
    ok = {k: v["ms"] for k, v in cells.items() if "ms" in v}
    return min(ok, key=ok.get) if ok else None


# ------------------------------------------------------------------------------ config 3
def grid_3d(comm: Comm, budget: Budget, shapes: Sequence[Tuple[int, int, int]] = GRID_3D,
            ops: Sequence[str] = GRID_3D_OPS, iters: int = 10) -> Dict:
    rows, skipped = [], []
    for shape in shapes:
        if budget.exhausted():
            skipped.append(list(shape))
            continue
        data = local_step(comm, lambda: make_data(shape, torch.bfloat16, comm.rank, comm.device))
        row = {"shape": list(shape), "bytes_per_rank": data.numel() * data.element_size()}
        for op_name in ops:
            cells = {label: _measure(comm, op_name, shape, data, label, opts, iters)
                     for label, opts in _candidates(comm)}
            best = _best(cells)
            row[op_name] = {"by_impl": cells, "best": best,
                            "busbw_GBps": cells[best]["busbw_GBps"] if best else None}
        rows.append(row)
        del data
        if comm.is_gpu:
            torch.cuda.empty_cache()
    return {"what": "3D activation-shaped all-gather + reduce-scatter (BASELINE config 3), bf16, "
                    "mean of back-to-back calls, rank max; busBW nccl-tests convention",
            "world": comm.world_size, "rows": rows,
            **({"skipped_budget": skipped} if skipped else {})}


# ------------------------------------------------------------------------------ config 4
def moe_alltoall(comm: Comm, budget: Budget, payloads: Sequence[Tuple[int, int]] = MOE_PAYLOADS,
                 iters: int = 10) -> Dict:
    rows, skipped = [], []
    for tokens, hidden in payloads:
        if budget.exhausted():
            skipped.append([tokens, hidden])
            continue
        shape = (tokens, hidden)
        data = local_step(comm, lambda: make_data(shape, torch.bfloat16, comm.rank, comm.device))
        cells = {label: _measure(comm, "alltoall_moe", shape, data, label, opts, iters)
                 for label, opts in _candidates(comm)}
        best = _best(cells)
        rows.append({"tokens_per_rank": tokens, "hidden": hidden,
                     "bytes_per_rank": data.numel() * data.element_size(),
                     "by_impl": cells, "best": best,
                     "busbw_GBps": cells[best]["busbw_GBps"] if best else None})
        del data
    return {"what": "MoE expert-parallel dispatch: uneven all-to-all, Zipf-skewed top-k router "
                    "splits (parallel.collectives.moe_split_sizes; BASELINE config 4), bf16",
            "world": comm.world_size, "rows": rows,
            **({"skipped_budget": skipped} if skipped else {})}


# ------------------------------------------------------------------------------ config 5
def ddp_candidates(comm: Comm) -> List[str]:
    if comm.world_size == 1 or not comm.is_gpu:
        return ["rccl"]                     # world 1 / CPU: the process-group path only
    # most likely fastest first: the time box may cut the tail of this list at P = 8
    return ["auto", "native", "custom", "rccl"]


def gpt2_ddp(comm: Comm, budget: Budget, steps: int = 10, warmup: int = 3,
             model: Optional[Dict] = None, candidates: Optional[Sequence[str]] = None) -> Dict:
    """GPT-2 DDP step per bucket all-reduce path; the fastest on rank-max ms/step is ``best``.
    Each candidate is a full training run (fresh model, same seed): warmup steps, then ``steps``
    timed steps between [barrier + sync] and [sync], plus one more step with comm events for
    the exposed-comm report."""
    from ..cli.train_ddp import parse_args, run

    m = dict(GPT2_SMALL, **(model or {}))
    comm.install_tune_agreement()           # GEMM choices agreed on rank-max timings
    by, skipped = {}, []
    for cand in (candidates or ddp_candidates(comm)):
        if by and budget.exhausted():
            skipped.append(cand)
            continue
        argv = ["--n-layer", str(m["n_layer"]), "--n-head", str(m["n_head"]),
                "--n-embd", str(m["n_embd"]), "--vocab", str(m["vocab"]),
                "--batch", str(m["batch"]), "--seq", str(m["seq"]), "--steps", str(steps),
                "--warmup", str(warmup), "--allreduce", cand]
        if comm.is_gpu:
            argv.append("--comm-timeline")      # HIP events around each bucket reduction
        err, res = None, None
        try:
            res = run(parse_args(argv), comm, overlap=True)
        except Exception as e:  # noqa: BLE001 - one path failing does not drop the others
            err = f"{type(e).__name__}: {e}"[:500]
        bad = _agree_errors(comm, err)
        if bad:
            by[cand] = {"error": bad[min(bad)]}
            if comm.is_gpu:
                torch.cuda.empty_cache()
            continue
        tail = res.get("comm_tail") or {}
        by[cand] = {"ms_per_step": round(res["ms_per_step"], 4),
                    "tokens_per_s": round(res["tokens_per_s"], 1),
                    "tflops_per_gpu": round(res["tflops_per_gpu"], 2),
                    "loss_first_step": res["loss_first_step"], "loss": res["loss"],
                    "buckets": res["buckets"],
                    "bucket_paths": res.get("bucket_paths"),
                    "exposed_comm_ms": tail.get("exposed_comm_ms"),
                    "bytes_reduced_after_backward": tail.get("bytes_reduced_after_backward"),
                    "hand_written_time_fraction":
                        res["gemm_kernel_mix"].get("hand_written_time_fraction"),
                    "gemm_tune_timing": res.get("gemm_tune_timing")}
    ok = {k: v["ms_per_step"] for k, v in by.items() if "ms_per_step" in v}
    best = min(ok, key=ok.get) if ok else None
    out = {"what": "GPT-2 DDP training step (BASELINE config 5): forward, backward with bucketed "
                   "gradient all-reduce overlapped, fused AdamW; synthetic tokens, random init",
           "model": f"gpt2 L{m['n_layer']} H{m['n_embd']} heads{m['n_head']} V{m['vocab']}",
           "batch_per_gpu": m["batch"], "seq_len": m["seq"],
           "global_batch": m["batch"] * comm.world_size, "world": comm.world_size,
           "steps": steps, "warmup": warmup, "by_allreduce": by, "best": best}
    if best:
        out.update(ms_per_step=by[best]["ms_per_step"], tokens_per_s=by[best]["tokens_per_s"])
    if skipped:
        out["skipped_budget"] = skipped
    return out
