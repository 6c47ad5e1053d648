"""Diagnostic: where does the round-2 DDP configuration (no late bucket, one AdamW pass) stall
the compute stream behind the comm stream? Events on the compute stream at step start, forward
end, every bucket launch (and whether the launch came from a backward hook or after backward),
backward end and step end, for split optimizer off / on, at one emulated bus bandwidth."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from distributed_llm_backend_benchmark_amd.data import SyntheticTokenDataset  # noqa: E402
from distributed_llm_backend_benchmark_amd.models.gpt2 import GPT2, GPT2Config  # noqa: E402
from distributed_llm_backend_benchmark_amd.parallel import ddp  # noqa: E402

gbps = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
dev = torch.device("cuda", 0)
cfg = GPT2Config(vocab_size=50304, block_size=1024, n_layer=12, n_head=12, n_embd=768)
for split in (False, True, False, True):
    model = GPT2(cfg, device=dev)
    tr = ddp.FlatParamTrainer(model, None, emulate_comm=gbps, late_bucket=False,
                              split_optimizer=split)
    data = SyntheticTokenDataset(16, 1024, cfg.vocab_size, device=dev)
    marks = []
    orig = tr._launch

    def launch(b, _orig=orig):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        marks.append((f"launch{b.idx}", ev, torch.autograd.graph.current_graph_task_id()
                      if hasattr(torch.autograd.graph, "current_graph_task_id") else None,
                      time.perf_counter()))
        _orig(b)
    tr._launch = launch
    for _ in range(4):
        x, y = data.get_batch()
        tr.step(x, y, sync_loss=False)
    torch.cuda.synchronize()
    marks.clear()
    x, y = data.get_batch()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    tr.timeline = True
    loss = tr.step(x, y, sync_loss=False)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev1.record()
    torch.cuda.synchronize()
    rep = tr.comm_tail_report()
    bwd = tr._tl_last["bwd_end"]
    out = {"split": split, "step_ms": round(ev0.elapsed_time(ev1), 3),
           "bwd_end_ms": round(ev0.elapsed_time(bwd), 3),
           "launch_points_ms": [(m[0], round(ev0.elapsed_time(m[1]), 3), m[2]) for m in marks],
           "comm": [(r["bucket"], round(r["start_ms"], 3), round(r["end_ms"], 3))
                    for r in rep["buckets"]]}
    print(json.dumps(out), flush=True)
    tr.close()
    del tr, model
