"""What overlapped gradient reduction costs the GPT-2 backward pass on ONE MI355X.

At world 1 the DDP trainer has no peers, so its bucket all-reduces never run. Here every ready
bucket instead launches a stand-in reduction on the high-priority comm stream at its
bucket-ready hook (``FlatParamTrainer(emulate_comm=True)``: bucket + zeros -> bucket, i.e. the
local HBM traffic of one rank's all-reduce — read 2n, write n — gradients unchanged), with a CU
budget of ``comm_blocks`` workgroups per launch. Compared: the step with no reduction
(baseline), overlapped reductions for bucket_mb x comm_blocks, and the same reductions
serialized after backward (overlap off). Each setting: fresh model, warmup, timed steps; the
baseline is measured first and last.

usage: python tools/ddp_overlap.py --out profiles/r02_overlap/ddp_overlap.jsonl
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--buckets", default="16,32,64")
    ap.add_argument("--blocks", default="8,32,128,256,0", help="0 = kernel heuristic")
    args = ap.parse_args(argv)

    from distributed_llm_backend_benchmark_amd.cli import train_ddp
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("rccl")
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    fh = open(args.out, "w")

    def one(label, bucket_mb, blocks, emulate, overlap):
        a = train_ddp.parse_args(["--steps", str(args.steps), "--warmup", str(args.warmup),
                                  "--bucket-mb", str(bucket_mb)]
                                 + (["--emulate-comm"] if emulate else [])
                                 + (["--comm-blocks", str(blocks)] if blocks else []))
        res = train_ddp.run(a, comm, overlap=overlap)
        rec = {"label": label, "bucket_mb": bucket_mb, "comm_blocks": blocks or None,
               "emulate_comm": emulate, "overlap": overlap, "buckets": res["buckets"],
               "ms_per_step": round(res["ms_per_step"], 4),
               "tokens_per_s": round(res["tokens_per_s"], 1), "loss": res["loss"]}
        print(json.dumps(rec), flush=True)
        fh.write(json.dumps(rec) + "\n")
        fh.flush()
        return rec

    base0 = one("baseline", 64, 0, False, True)
    rows = []
    for bmb in [float(x) for x in args.buckets.split(",")]:
        for nb in [int(x) for x in args.blocks.split(",")]:
            rows.append(one("overlapped", bmb, nb, True, True))
    rows.append(one("serialized", 64, 0, True, False))
    base1 = one("baseline", 64, 0, False, True)
    base = min(base0["ms_per_step"], base1["ms_per_step"])
    for r in rows:
        r["slowdown_pct_vs_baseline"] = round(100.0 * (r["ms_per_step"] / base - 1.0), 2)
        fh.write(json.dumps({"summary": True, **r}) + "\n")
    fh.close()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
