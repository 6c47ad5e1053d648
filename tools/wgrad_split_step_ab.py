"""GPT-2 DDP step (world 1) A/B of the weight-gradient split-K cap, VERDICT r05 item 4.

The default split fills about one resident wave when the dW kernel has the chip; in the step it
runs on the side stream beside the main stream's backward, where its fp32 partials (tens of MB
per dW, written then re-read by the reduce pass) compete for HBM. Caps 1 / 2 / 4 / none,
interleaved, ``--reps`` rounds, one process (each run builds a fresh trainer; the autotuner's
per-shape choices are re-made per cap). One JSON line per run.

    python tools/wgrad_split_step_ab.py --reps 2 --caps none,4,2,1
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--caps", default="none,4,2,1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()

    from distributed_llm_backend_benchmark_amd.cli import train_ddp
    from distributed_llm_backend_benchmark_amd.ops import gemm
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed

    comm = init_distributed("auto")
    args = train_ddp.parse_args(["--steps", str(a.steps), "--warmup", str(a.warmup)])
    caps = [None if c == "none" else int(c) for c in a.caps.split(",")]
    for rep in range(a.reps):
        for cap in caps:
            gemm.set_wgrad_split_cap(cap)
            gemm.WGRAD_CHOICES.clear()
            res = train_ddp.run(args, comm, overlap=True)
            print(json.dumps({"rep": rep, "split_cap": cap, "ms_per_step": res["ms_per_step"],
                              "side_stream_checks": res["side_stream_checks"],
                              "wgrad_choices": {str(k[:3]): v for k, v in
                                                gemm.WGRAD_CHOICES.items()}}), flush=True)
    gemm.set_wgrad_split_cap(None)
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
