"""A/B of the causal attention forward's workgroup shape: waves per
workgroup (4: 128 queries; 8: 256 queries sharing each K/V tile — half the DMA, barriers and
workgroup prologues per FLOP) x K/V ring depth (2 tiles with builtin LDS reads; 3 tiles with asm
reads and counted waits, so the next tile's DMA stays in flight across a tile). Interleaved
rounds, best of ``--rounds``; every shape's output checked bit-identical to the (4, 2) default.

    python tools/attn_fwd_shape_ab.py [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402
from distributed_llm_backend_benchmark_amd.ops.attention import attn_fwd  # noqa: E402

SHAPES = ((4, 2), (8, 2), (4, 3), (8, 3))
CASES = ((16, 1024, 12, 64), (8, 2048, 12, 64), (4, 4096, 16, 64), (16, 1024, 6, 128),
         (4, 4096, 8, 128))


def t_us(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    lib = _lib.lib()
    for B, T, H, D in CASES:
        qkv = torch.randn(B, T, 3 * H * D, device="cuda").to(torch.bfloat16)
        lib.dlbb_attn_set_fwd_shape(4, 2)
        ref_o, ref_l = attn_fwd(qkv, H)
        same = {}
        for nw, ns in SHAPES:
            lib.dlbb_attn_set_fwd_shape(nw, ns)
            o, lse = attn_fwd(qkv, H)
            same[f"{nw}x{ns}"] = bool(torch.equal(o, ref_o) and torch.equal(lse, ref_l))
        best = {f"{nw}x{ns}": 1e9 for nw, ns in SHAPES}
        for _ in range(a.rounds):
            for nw, ns in SHAPES:
                lib.dlbb_attn_set_fwd_shape(nw, ns)
                k = f"{nw}x{ns}"
                best[k] = min(best[k], t_us(lambda: attn_fwd(qkv, H)))
        lib.dlbb_attn_set_fwd_shape(4, 2)
        fl = 4.0 * B * H * T * T * D / 2
        print(json.dumps({"B": B, "T": T, "H": H, "D": D, "us": {k: round(v, 2) for k, v in
                                                                 best.items()},
                          "tflops": {k: round(fl / v / 1e6, 1) for k, v in best.items()},
                          "bit_identical_to_4x2": same}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
