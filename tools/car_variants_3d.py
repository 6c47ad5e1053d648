"""IPC all-reduce ALGORITHM variants on the reference's variant grid, single-GPU emulation.

The reference sweeps oneCCL's all-reduce algorithm (``CCL_ALLREDUCE`` in
``collectives/3d/launch_dsccl.sh:46-47``) on B in {8, 16} x S in {2048, 4096} x H in {2048,
4096} bf16 at 4 and 8 ranks and keeps one result directory per algorithm
(``collectives/3d/results/dsccl_<algo>_allreduce``). This tool produces the same layout for our
algorithms — one-shot, staged two-shot, registered in-place two-shot (pull) and its push form —
with W virtual ranks on ONE MI355X (:mod:`...parallel.virtual_ranks`; every byte moves through
one HBM, not xGMI: protocol + memory-level-parallelism numbers, labelled as such in every file).
Reference warmup / iteration counts (10 / 100); each iteration is timed with a device event pair
and every rank's entry is that fused launch's time; each configuration is validated against an
fp32 sum first. Then ``cli.stats --mode 3d`` gives the reference's standard / transposed CSVs.

usage: python tools/car_variants_3d.py --out results/vr_custom
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_llm_backend_benchmark_amd.bench.schema import filename_3d, result_3d  # noqa: E402
from distributed_llm_backend_benchmark_amd.parallel import virtual_ranks as vr  # noqa: E402

VARIANTS = {"oneshot": vr.K_ONESHOT, "twoshot": vr.K_TWOSHOT, "reg_pull": vr.K_REG,
            "reg_push": vr.K_PUSH}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", required=True)
    ap.add_argument("--worlds", default="4,8")
    ap.add_argument("--batch-sizes", default="8,16")
    ap.add_argument("--seq-lengths", default="2048,4096")
    ap.add_argument("--hidden-dims", default="2048,4096")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args(argv)
    dev = torch.device("cuda", torch.cuda.current_device())
    shapes = [(b, s, h) for b in map(int, args.batch_sizes.split(","))
              for s in map(int, args.seq_lengths.split(","))
              for h in map(int, args.hidden_dims.split(","))]
    cap = max(b * s * h * 2 for b, s, h in shapes)
    for W in map(int, args.worlds.split(",")):
        V = vr.VirtualRanks(W, capacity_bytes=cap)
        try:
            for name, kind in VARIANTS.items():
                impl = f"vr_custom_{name}_allreduce"
                odir = os.path.join(args.out, impl)
                os.makedirs(odir, exist_ok=True)
                nb = min(V.max_blocks(kind), 256 if kind in (vr.K_REG, vr.K_PUSH) else 128)
                for B, S, H in shapes:
                    n = B * S * H
                    xs = []
                    for r in range(W):
                        g = torch.Generator(device=dev)
                        g.manual_seed(42 + r)            # reference: torch.manual_seed(42 + rank)
                        xs.append(torch.randn(n, generator=g, device=dev).to(torch.bfloat16))
                    ref = sum(x.float() for x in xs)
                    reg = kind in (vr.K_REG, vr.K_PUSH)
                    if reg:
                        bufs = [x.clone() for x in xs]
                        rid = V.register(bufs)
                        fn = lambda: V.all_reduce_registered(bufs, rid, nblocks=nb,  # noqa: E731
                                                             push=kind == vr.K_PUSH)
                        fn()
                        got = bufs
                    else:
                        outs = [torch.empty_like(x) for x in xs]
                        fn = lambda: V.all_reduce(xs, outs, algo=kind, nblocks=nb)  # noqa: E731
                        fn()
                        got = outs
                    torch.cuda.synchronize()
                    ok = not any(V.errors()) and all(
                        torch.allclose(t.float(), ref, rtol=2e-2, atol=5e-2 * W) for t in got)
                    del ref
                    if not ok:
                        print(json.dumps({"impl": impl, "W": W, "shape": [B, S, H],
                                          "valid": False}), flush=True)
                        continue
                    if reg:
                        for t in bufs:
                            t.zero_()          # in-place sums grow W x per call
                    for _ in range(args.warmup):
                        fn()
                    evs = [(torch.cuda.Event(enable_timing=True),
                            torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
                    for a, b in evs:
                        a.record()
                        fn()
                        b.record()
                    torch.cuda.synchronize()
                    t = [a.elapsed_time(b) * 1e-3 for a, b in evs]
                    rec = result_3d(impl=impl, backend="virtual_ranks_one_gpu", op="allreduce",
                                    ranks=W, batch=B, seq_len=S, hidden_dim=H, dtype="bfloat16",
                                    wire_dtype="bfloat16", wire_bytes=n * 2, warmup=args.warmup,
                                    iters=args.iters, timing_method="hip_event_fused_launch",
                                    timings=[list(t) for _ in range(W)],
                                    extra={"nblocks": nb, "validated": True,
                                           "emulation": "W ranks on ONE MI355X (one fused "
                                                        "launch; traffic through one HBM, not "
                                                        "xGMI)",
                                           "errors_after": V.errors()})
                    with open(os.path.join(odir, filename_3d(impl, "allreduce", W, B, S, H)),
                              "w") as f:
                        json.dump(rec, f)
                    med = sorted(t)[len(t) // 2]
                    print(json.dumps({"impl": impl, "W": W, "shape": [B, S, H], "nblocks": nb,
                                      "p50_ms": round(med * 1e3, 4), "valid": True}), flush=True)
                    del xs, got
                    if reg:
                        del bufs
                    else:
                        del outs
        finally:
            V.close()
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
