"""The DDP gradient-sync tail on ONE MI355X, link-bound.

Every bucket-ready hook launches a stand-in all-reduce on the comm stream: the local HBM traffic
of one rank's all-reduce plus a spin that lasts the ring all-reduce time of the bucket at an
assumed xGMI bus bandwidth over ``--world`` ranks (``FlatParamTrainer(emulate_comm=<GB/s>)``).
Per bandwidth, two layouts of the same GPT-2 step:

* ``before`` — round 2: buckets closed by size only (the last bucket = blocks 1-0 + the tied
  77 MB wte + wpe, ready only after the embedding backward), one AdamW after every reduction;
* ``after``  — the embedding tables in a bucket of their own and AdamW split around it (the
  other buckets' update runs while the tail bucket is still being reduced).

Reported per run: ms/step, bytes whose reduction started after backward ended, exposed comm
time (last reduction end - backward end) and the optimizer's end, from one step with events.

usage: python tools/ddp_tail.py --out profiles/r03_overlap/ddp_tail.jsonl
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", required=True)
    ap.add_argument("--gbps", default="50,100,300")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    args = ap.parse_args(argv)

    from distributed_llm_backend_benchmark_amd.cli import train_ddp
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("rccl")
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    fh = open(args.out, "w")

    def one(label, gbps, before):
        argv_ = ["--steps", str(args.steps), "--warmup", str(args.warmup),
                 "--bucket-mb", str(args.bucket_mb), "--emulate-world", str(args.world),
                 "--comm-timeline"]
        if gbps:
            argv_ += ["--emulate-comm", str(gbps)]
        if before:
            argv_ += ["--no-late-bucket", "--no-split-optimizer"]
        res = train_ddp.run(train_ddp.parse_args(argv_), comm, overlap=True)
        tail = res.get("comm_tail") or {}
        rec = {"label": label, "busbw_GBps": gbps, "world": args.world,
               "ms_per_step": round(res["ms_per_step"], 4), "buckets": res["buckets"],
               "bytes_reduced_after_backward": tail.get("bytes_reduced_after_backward"),
               "exposed_comm_ms": tail.get("exposed_comm_ms"),
               "optimizer_end_ms_after_backward": tail.get("optimizer_end_ms"),
               "bucket_timeline": tail.get("buckets")}
        print(json.dumps({k: v for k, v in rec.items() if k != "bucket_timeline"}), flush=True)
        fh.write(json.dumps(rec) + "\n")
        fh.flush()
        return rec

    base = [one("no_comm", None, False)]
    for g in [float(x) for x in args.gbps.split(",")]:
        one("before", g, True)
        one("after", g, False)
    base.append(one("no_comm", None, False))
    fh.write(json.dumps({"baseline_ms": min(b["ms_per_step"] for b in base)}) + "\n")
    fh.close()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
