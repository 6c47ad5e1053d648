"""Measure the IPC xGMI collective kernels on ONE MI355X with W virtual ranks
(:mod:`distributed_llm_backend_benchmark_amd.parallel.virtual_ranks`).

Sections (one JSON line per configuration, every configuration validated once against an fp32
sum of the W rank inputs before it is timed; a configuration that fails is recorded with
``"valid": false`` and never timed):

* ``latency``    one-shot all-reduce, 512 B .. 256 KiB, workgroups per rank swept
* ``crossover``  one-shot vs staged two-shot vs registered two-shot, 64 KiB .. 8 MiB
* ``throughput`` staged two-shot, registered in-place two-shot (pull) and push form,
                 1 MiB .. 128 MiB, workgroups per rank swept
* ``direct``     one-hop all-gather / reduce-scatter / all-to-all on registered inputs
* ``streams``    the per-rank production launch on W streams (W concurrent kernels), W = 2, 4

Times: ``us_b2b`` = mean per call of ``iters`` back-to-back launches between two events (the
nccl-tests convention); ``us_p50`` = median of per-call event pairs. ``hbm_GBps`` = the bytes the
W ranks together load + store per call (model in ``_hbm_bytes``) / time: on one GPU every byte a
real rank would move over xGMI goes through this GPU's memory system, so large messages are
bounded by the HBM roofline (~8 TB/s; messages that fit L2 / the 256 MB MALL can exceed it), not
by xGMI; small messages give the protocol's latency floor.

usage: python tools/car_harness.py --out profiles/r02_car_harness/car_harness.jsonl [--quick]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_llm_backend_benchmark_amd.parallel import virtual_ranks as vr  # noqa: E402

BF16 = torch.bfloat16


def _hbm_bytes(kind: int, n: int, W: int) -> int:
    """HBM bytes read + written per call by all W ranks together (message n bytes per rank)."""
    s = n // W
    per_rank = {
        vr.K_ONESHOT: 2 * n + W * n + n,                       # copy-in r+w, W reads, 1 write
        vr.K_TWOSHOT: 2 * n + W * s + 2 * s + 2 * (W - 1) * s,  # copy-in, RS (tmp+out), AG
        vr.K_REG: W * s + s + 2 * (W - 1) * s,                  # RS in place, AG pulls
        vr.K_PUSH: 2 * n + W * s + W * s,                       # push-in, reduce, push-out
        vr.K_AG: 2 * W * n,                                     # n = chunk per rank
        vr.K_A2A: 2 * n,                                        # n = whole input per rank
        vr.K_RS: W * s + s,
    }[kind]
    return W * per_rank


def _rank_data(W: int, numel: int, seed: int, dev) -> list:
    out = []
    for r in range(W):
        g = torch.Generator(device=dev)
        g.manual_seed(seed + r)
        out.append(torch.randn(numel, generator=g, device=dev).to(BF16))
    return out


def _close(got: torch.Tensor, exp: torch.Tensor, W: int) -> bool:
    return bool(torch.allclose(got.float(), exp.float(), rtol=2e-2, atol=5e-2 * W))


def _time(fn, iters: int, stream) -> tuple:
    """(mean us per call back to back, p50 us of per-call event pairs)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(iters):
        fn()
    e.record(stream)
    torch.cuda.synchronize()
    b2b = s.elapsed_time(e) * 1e3 / iters
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(min(iters, 50))]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    p50 = statistics.median(a.elapsed_time(b) * 1e3 for a, b in evs)
    return b2b, p50


class Harness:
    def __init__(self, out, quick: bool):
        self.out = out
        self.quick = quick
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.stream = torch.cuda.current_stream()

    def emit(self, rec: dict) -> None:
        rec["device"] = torch.cuda.get_device_name(self.dev)
        line = json.dumps(rec)
        print(line, flush=True)
        self.out.write(line + "\n")
        self.out.flush()

    # -------------------------------------------------------------- all-reduce (fused form)
    def allreduce(self, section, V, kind, nbytes, blocks, iters):
        W = V.world
        numel = nbytes // 2
        xs = _rank_data(W, numel, 11 * nbytes + kind, self.dev)
        ref = sum(x.float() for x in xs)
        reg = kind in (vr.K_REG, vr.K_PUSH)
        if reg:
            bufs = [x.clone() for x in xs]
            rid = V.register(bufs)
        else:
            outs = [torch.empty_like(x) for x in xs]
        for nb in blocks:
            if nb > V.max_blocks(kind):
                continue
            rec = {"section": section, "kind": vr.KIND_NAMES[kind], "world": W, "bytes": nbytes,
                   "nblocks": nb, "form": "fused"}
            if reg:
                for b, x in zip(bufs, xs):
                    b.copy_(x)
                V.all_reduce_registered(bufs, rid, nblocks=nb, push=kind == vr.K_PUSH)
                got = bufs
            else:
                V.all_reduce(xs, outs, algo=kind, nblocks=nb)
                got = outs
            torch.cuda.synchronize()
            errs = V.errors()
            rec["valid"] = all(_close(g, ref, W) for g in got) and not any(errs)
            if not rec["valid"]:
                rec["errors"] = errs
                self.emit(rec)
                continue
            if reg:
                for b in bufs:          # bounded values while timing (in place sums grow W x)
                    b.zero_()
                fn = lambda: V.all_reduce_registered(bufs, rid, nblocks=nb,  # noqa: E731
                                                     push=kind == vr.K_PUSH)
            else:
                fn = lambda: V.all_reduce(xs, outs, algo=kind, nblocks=nb)  # noqa: E731
            b2b, p50 = _time(fn, iters, self.stream)
            errs = V.errors()
            rec.update(us_b2b=round(b2b, 3), us_p50=round(p50, 3), timing_errors=any(errs),
                       hbm_GBps=round(_hbm_bytes(kind, nbytes, W) / (b2b * 1e-6) / 1e9, 1))
            self.emit(rec)

    # -------------------------------------------------------------- direct kernels
    def direct(self, V, kind, nbytes, blocks, iters):
        """nbytes = registered input per rank."""
        W = V.world
        numel = nbytes // 2
        xs = _rank_data(W, numel, 7 * nbytes + kind, self.dev)
        rid = V.register(xs)
        if kind == vr.K_AG:
            outs = [torch.empty(W * numel, dtype=BF16, device=self.dev) for _ in range(W)]
            exp = [torch.cat(xs) for _ in range(W)]
        elif kind == vr.K_A2A:
            outs = [torch.empty(numel, dtype=BF16, device=self.dev) for _ in range(W)]
            c = numel // W
            exp = [torch.cat([x[r * c:(r + 1) * c] for x in xs]) for r in range(W)]
        else:
            outs = [torch.empty(numel // W, dtype=BF16, device=self.dev) for _ in range(W)]
            tot = sum(x.float() for x in xs)
            exp = list(tot.chunk(W))
        for nb in blocks:
            if nb > V.max_blocks(kind):
                continue
            rec = {"section": "direct", "kind": vr.KIND_NAMES[kind], "world": W,
                   "bytes": nbytes, "nblocks": nb, "form": "fused"}
            for o in outs:
                o.zero_()
            V.direct(kind, xs, rid, outs, nblocks=nb)
            torch.cuda.synchronize()
            errs = V.errors()
            rec["valid"] = all(_close(o, e, W) for o, e in zip(outs, exp)) and not any(errs)
            if rec["valid"]:
                b2b, p50 = _time(lambda: V.direct(kind, xs, rid, outs, nblocks=nb), iters,
                                 self.stream)
                chunk = nbytes if kind == vr.K_AG else nbytes
                rec.update(us_b2b=round(b2b, 3), us_p50=round(p50, 3),
                           timing_errors=any(V.errors()),
                           hbm_GBps=round(_hbm_bytes(kind, chunk, W) / (b2b * 1e-6) / 1e9, 1))
            else:
                rec["errors"] = errs
            self.emit(rec)

    # -------------------------------------------------------------- per-rank streams
    def streams(self, W, kind, nbytes, nb, iters):
        V = vr.VirtualRanks(W, capacity_bytes=max(nbytes, 1 << 20))
        try:
            sts = [torch.cuda.Stream(priority=-1) for _ in range(W)]
            xs = _rank_data(W, nbytes // 2, 3 * nbytes, self.dev)
            outs = [torch.empty_like(x) for x in xs]
            ref = sum(x.float() for x in xs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            V.all_reduce_streams(xs, outs, sts, algo=kind, nblocks=nb)
            torch.cuda.synchronize()
            first_s = time.perf_counter() - t0
            errs = V.errors()
            rec = {"section": "streams", "kind": vr.KIND_NAMES[kind], "world": W,
                   "bytes": nbytes, "nblocks": nb, "form": "streams",
                   "first_call_s": round(first_s, 4)}
            rec["valid"] = all(_close(o, ref, W) for o in outs) and not any(errs)
            if not rec["valid"]:
                rec["errors"] = errs
                self.emit(rec)
                return False
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                V.all_reduce_streams(xs, outs, sts, algo=kind, nblocks=nb)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            rec.update(us_host_per_call=round(dt * 1e6, 3), timing_errors=any(V.errors()))
            self.emit(rec)
            return True
        finally:
            V.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", required=True)
    ap.add_argument("--quick", action="store_true", help="fewer sizes / block counts")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--sections", default="latency,crossover,throughput,direct,streams")
    args = ap.parse_args(argv)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    worlds = [int(w) for w in args.worlds.split(",")]
    sections = set(args.sections.split(","))
    with open(args.out, "w") as fh:
        H = Harness(fh, args.quick)
        lat_sizes = [512, 4096, 32 << 10, 256 << 10] if args.quick else \
            [512, 2048, 8192, 32 << 10, 128 << 10, 256 << 10]
        big = [1 << 20, 16 << 20, 128 << 20] if args.quick else \
            [1 << 20, 4 << 20, 16 << 20, 64 << 20, 128 << 20]
        for W in worlds:
            V = vr.VirtualRanks(W, capacity_bytes=128 << 20)
            try:
                if "latency" in sections:
                    for n in lat_sizes:
                        H.allreduce("latency", V, vr.K_ONESHOT, n, [1, 2, 4, 8, 16, 32],
                                    iters=200)
                if "crossover" in sections:
                    # one-shot vs staged two-shot vs registered two-shot around the crossovers
                    for n in [64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20,
                              8 << 20]:
                        for kind in (vr.K_ONESHOT, vr.K_TWOSHOT, vr.K_REG):
                            H.allreduce("crossover", V, kind, n, [4, 8, 16, 32, 64, 128],
                                        iters=100)
                if "throughput" in sections:
                    for n in big:
                        for kind in (vr.K_TWOSHOT, vr.K_REG, vr.K_PUSH):
                            H.allreduce("throughput", V, kind, n, [32, 64, 128, 256],
                                        iters=50 if n <= 16 << 20 else 10)
                if "direct" in sections:
                    for n in ([1 << 20, 16 << 20] if args.quick else [1 << 20, 8 << 20, 64 << 20]):
                        for kind in (vr.K_AG, vr.K_RS, vr.K_A2A):
                            H.direct(V, kind, n, [32, 64, 128, 256],
                                     iters=50 if n <= 8 << 20 else 10)
            finally:
                V.close()
        if "streams" in sections:
            for W in (2, 4):
                for kind, n, nb in ((vr.K_ONESHOT, 4096, 4), (vr.K_ONESHOT, 256 << 10, 16),
                                    (vr.K_TWOSHOT, 16 << 20, 64)):
                    if not H.streams(W, kind, n, nb, iters=20):
                        break       # a serialized pair of queues: the rest would time out too
    return 0


if __name__ == "__main__":
    sys.exit(main())
