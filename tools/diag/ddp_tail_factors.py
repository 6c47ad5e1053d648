"""Diagnostic: DDP tail timeline for (late bucket on/off) x (split optimizer on/off), repeated,
at one emulated bus bandwidth — separates the two factors of tools/ddp_tail.py."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from distributed_llm_backend_benchmark_amd.cli import train_ddp  # noqa: E402
from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed  # noqa: E402

gbps = sys.argv[1] if len(sys.argv) > 1 else "300"
comm = init_distributed("rccl")
for rep in range(2):
    for late in (False, True):
        for split in (False, True):
            argv = ["--steps", "8", "--warmup", "3", "--emulate-comm", gbps, "--comm-timeline"]
            if not late:
                argv.append("--no-late-bucket")
            if not split:
                argv.append("--no-split-optimizer")
            res = train_ddp.run(train_ddp.parse_args(argv), comm, overlap=True)
            t = res["comm_tail"]
            print(json.dumps({"rep": rep, "late": late, "split": split,
                              "ms": round(res["ms_per_step"], 3),
                              "opt_end": t["optimizer_end_ms"],
                              "buckets": [(b["bytes"] >> 20, b["start_ms"], b["end_ms"])
                                          for b in t["buckets"]]}), flush=True)
comm.destroy()
