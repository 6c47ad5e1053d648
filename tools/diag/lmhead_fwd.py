"""GPT-2 LM-head forward (16384 x 50304 x 768) on the persistent ping-pong: balanced vs plain DMA
issue, with and without the C stores (diagnostic no-store build path), vs hipBLASLt; interleaved
rounds, best-of. One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_backend_benchmark_amd.ops import _lib, linear  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.gemm import set_bal  # noqa: E402

M, N, K = 16384, 50304, 768
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
lib = _lib.lib()


def run(cfg):
    os.environ["DLBB_GEMM"] = "blas" if cfg == "blas" else "mfma"
    set_bal(1 if cfg.startswith("bal") else 0 if cfg.startswith("plain") else 2)
    lib.dlbb_gemm_set_diag_nostore(1 if cfg.endswith("nostore") else 0)
    return linear(x, w)


cfgs = ["default", "plain", "bal", "plain_nostore", "bal_nostore", "blas"]
best = {c: 1e9 for c in cfgs}
for _ in range(5):
    for c in cfgs:
        run(c)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run(c)
        e.record()
        e.synchronize()
        best[c] = min(best[c], s.elapsed_time(e) / 10)
lib.dlbb_gemm_set_diag_nostore(0)
set_bal(2)
os.environ["DLBB_GEMM"] = "auto"
print(json.dumps({"shape": [M, N, K], "ms": {c: round(v, 4) for c, v in best.items()}}), flush=True)
