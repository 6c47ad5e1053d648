"""Root-cause probe of the high-priority overlap trap.

Round 2 measured +61-64 % GPT-2 step time with the bucket stand-in reduction on a HIGH-priority
comm stream at a few (bucket MiB, workgroups) settings, and the effect vanished under
rocprofv3's kernel trace. Here the same setting runs with per-workgroup start / end stamps
(``utils.stamps``: 32 bytes per workgroup, written after its last barrier — no dispatch
serialisation) on the six ping-pong GEMMs, the n-way reduction and the spin stand-in, for the
normal- and the high-priority stream back to back in one process. Per priority: ms/step (plain
timed steps), then one stamped step: per launch the dispatch spread (first -> last workgroup
start), the median / max workgroup duration, and which grids ran beside the comm kernels.

usage: python tools/overlap_trap.py --out profiles/r03_overlap/trap
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
    ap.add_argument("--bucket-mb", type=float, default=16.0)
    ap.add_argument("--blocks", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--prios", default="0,-1,0,-1")
    args = ap.parse_args(argv)

    import torch

    from distributed_llm_backend_benchmark_amd.cli import train_ddp
    from distributed_llm_backend_benchmark_amd.parallel import ddp
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.utils.stamps import Stamps, summarize

    os.environ["DLBB_ALLOW_HIGH_PRIO_COMM"] = "1"     # past the trainer's fence, on purpose
    comm = init_distributed("rccl")
    os.makedirs(args.out, exist_ok=True)
    fh = open(os.path.join(args.out, "trap_runs.jsonl"), "w")
    for k, prio in enumerate(int(p) for p in args.prios.split(",")):
        ddp._COMM_PRIORITY = prio
        a = train_ddp.parse_args(["--steps", str(args.steps), "--warmup", str(args.warmup),
                                  "--bucket-mb", str(args.bucket_mb), "--emulate-comm",
                                  "--comm-blocks", str(args.blocks)])
        res = train_ddp.run(a, comm, overlap=True)
        # one more step, stamped, on a fresh trainer state (same settings)
        from distributed_llm_backend_benchmark_amd.data import SyntheticTokenDataset
        from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config

        cfg = GPT2Config(vocab_size=a.vocab, block_size=a.seq, n_layer=a.n_layer,
                         n_head=a.n_head, n_embd=a.n_embd)
        model = GPT2(cfg, device=comm.device)
        tr = ddp.FlatParamTrainer(model, None, bucket_mb=a.bucket_mb, emulate_comm=True,
                                  comm_blocks=args.blocks)
        data = SyntheticTokenDataset(a.batch, a.seq, cfg.vocab_size, device=comm.device)
        for _ in range(2):
            x, y = data.get_batch()
            tr.step(x, y, sync_loss=False)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        x, y = data.get_batch()
        with Stamps(1 << 20) as st:
            s.record()
            tr.step(x, y, sync_loss=False)
            e.record()
        step_ms = s.elapsed_time(e)
        launches = st.collect()
        summ = summarize(launches)
        tr.close()
        del tr, model
        rec = {"run": k, "priority": prio, "bucket_mb": args.bucket_mb, "blocks": args.blocks,
               "ms_per_step": round(res["ms_per_step"], 4), "stamped_step_ms": round(step_ms, 4),
               "launches": summ}
        with open(os.path.join(args.out, f"stamps_run{k}_prio{prio}.json"), "w") as f:
            json.dump({"summary": summ, "launches": launches}, f)
        worst = sorted(summ, key=lambda r: -r["dispatch_spread_ns"])[:5]
        line = {"run": k, "priority": prio, "ms_per_step": rec["ms_per_step"],
                "stamped_step_ms": rec["stamped_step_ms"], "n_launches": len(summ),
                "worst_dispatch_spread": [(w["kind"], w["workgroups"],
                                           round(w["dispatch_spread_ns"] / 1e3, 1),
                                           round(w["median_wg_ns"] / 1e3, 1))
                                          for w in worst]}
        print(json.dumps(line), flush=True)
        fh.write(json.dumps(rec) + "\n")
        fh.flush()
    fh.close()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
