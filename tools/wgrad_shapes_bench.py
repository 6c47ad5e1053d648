"""Device time of the GPT-2 step's weight-gradient calls (the four per-layer dW shapes, each
with the fused bias gradient and bf16 accumulate, on the tile the step's autotuner picks) —
whole call incl. the split-K reduce, median of interleaved rounds. Run it once per tree to A/B
two builds (PYTHONPATH=<tree> python tools/wgrad_shapes_bench.py).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("PYTHONPATH", "").split(":")[0] or
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm as G  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops import _lib as _L  # noqa: E402,F401

SHAPES = (("qkv", 2304, 768, G._wgrad_hip_wide), ("proj", 768, 768, G._wgrad_hip256),
          ("fc", 3072, 768, G._wgrad_hip_wide), ("mproj", 768, 3072, G._wgrad_hip256))


def main():
    M = 16384
    g = torch.Generator(device="cuda").manual_seed(0)
    cases = []
    for name, N, K, fn in SHAPES:
        dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        b = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        cases.append((name, N, K, lambda fn=fn, dy=dy, x=x, w=w, b=b: fn(dy, x, w, True, None, b)))
    ts = {c[0]: [] for c in cases}
    for _ in range(7):
        for name, N, K, f in cases:
            f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                f()
            e.record()
            e.synchronize()
            ts[name].append(s.elapsed_time(e) * 1e3 / 20)
    out = {}
    for name, N, K, _ in cases:
        v = sorted(ts[name])[len(ts[name]) // 2]
        out[name] = {"us": round(v, 2), "tflops": round(2.0 * M * N * K / v / 1e6, 1)}
    out["lib"] = G._lib.LIB_PATH
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
