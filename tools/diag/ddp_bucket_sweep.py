"""Diagnostic: step time and post-backward comm tail vs bucket size, late bucket on/off, split
optimizer on, at emulated bus bandwidths (link-bound stand-in, P = 8)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from distributed_llm_backend_benchmark_amd.cli import train_ddp  # noqa: E402
from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed  # noqa: E402

comm = init_distributed("rccl")
for gbps in sys.argv[1].split(","):
    for mb in (16, 32, 64):
        for late in (False, True):
            argv = ["--steps", "8", "--warmup", "3", "--emulate-comm", gbps, "--comm-timeline",
                    "--bucket-mb", str(mb)]
            if not late:
                argv.append("--no-late-bucket")
            res = train_ddp.run(train_ddp.parse_args(argv), comm, overlap=True)
            t = res["comm_tail"]
            after = sum(b["bytes"] for b in t["buckets"] if b["end_ms"] > 0)
            print(json.dumps({"gbps": float(gbps), "bucket_mb": mb, "late": late,
                              "ms": round(res["ms_per_step"], 3), "buckets": res["buckets"],
                              "exposed_ms": t["exposed_comm_ms"], "opt_end": t["optimizer_end_ms"],
                              "bytes_in_flight_after_bwd": after}), flush=True)
comm.destroy()
