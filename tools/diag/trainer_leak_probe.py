"""Device memory across repeated in-process GPT-2 trainer builds (cli/train_ddp.run): after each
run, allocated / reserved bytes and the run's ms per step. Two of twenty in-process A/B runs took
10-13x longer (profiles/r06_step/SUMMARY.md); a leak that fills the 288 GB would do that (every
step then frees and re-allocates through the runtime, which synchronises).

    python tools/diag/trainer_leak_probe.py --runs 10
"""
import argparse
import gc
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch

    from distributed_llm_backend_benchmark_amd.cli import train_ddp
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("auto")
    args = train_ddp.parse_args(["--steps", str(a.steps), "--warmup", "3"])
    for i in range(a.runs):
        res = train_ddp.run(args, comm, overlap=True)
        gc.collect()
        torch.cuda.synchronize()
        st = torch.cuda.memory_stats()
        print(json.dumps({"run": i, "ms_per_step": round(res["ms_per_step"], 3),
                          "allocated_GB": round(torch.cuda.memory_allocated() / 2**30, 2),
                          "reserved_GB": round(torch.cuda.memory_reserved() / 2**30, 2),
                          "num_alloc_retries": st.get("num_alloc_retries", 0),
                          "num_device_alloc": st.get("num_device_alloc", 0)}), flush=True)
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
