"""Where a ping-pong NT workgroup's time goes (diagnostic): per-workgroup stamps at start, first
MFMA (prologue DMA landed), end of the K-loop and end of the C stores (``s_memrealtime``, one
100 MHz clock for the chip) for one plain bf16 GEMM. Prints per shape: kernel span, launch skew
(start spread), median prologue / loop / epilogue, loop time per K-tile, and the same for the
hipBLASLt kernel's wall time for reference.

    python tools/diag/pp_phases.py [--shapes 4096x4096x4096,...] [--nj 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from distributed_llm_backend_benchmark_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096x1024,4096x4096x4096,4096x4096x16384,"
                                        "16384x768x3072,4096x12288x4096")
    ap.add_argument("--nj", default="4")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    for spec in args.shapes.split(","):
        M, N, K = (int(v) for v in spec.split("x"))
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for nj in (int(v) for v in args.nj.split(",")):
            if nj == 3 and N % 192:
                continue
            tiles = -(-M // 256) * -(-N // (64 * nj))
            rec = torch.zeros(tiles * 4, dtype=torch.int64, device=dev)

            def run():
                _lib.check(lib.dlbb_gemm_nt_phase_probe(
                    x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), M, N,
                    K, nj, rec.data_ptr(), _lib.stream(dev)), "phase_probe")
            for _ in range(10):
                run()
            torch.cuda.synchronize()
            rows = []
            for _ in range(5):
                run()
                torch.cuda.synchronize()
                raw = rec.view(-1, 4).cpu()
                tag = (raw[:, 0] >> 48) & 0xFFFF
                raw = raw.clone()
                raw[:, 0] &= (1 << 48) - 1
                r = raw.double() * 10.0 / 1e3      # us
                t0 = r[:, 0].min()
                xcc = (tag >> 13) & 7
                loop = r[:, 2] - r[:, 1]
                per_xcc = {int(x): round(float(loop[xcc == x].median()), 2) for x in range(8)
                           if bool((xcc == x).any())}
                # loop time by tile position: workgroup b -> tile (XCD-aware remap in tile_of)
                rows.append({"span": float(r[:, 3].max() - t0),
                             "skew": float(r[:, 0].max() - t0),
                             "pro": float((r[:, 1] - r[:, 0]).median()),
                             "loop": float((r[:, 2] - r[:, 1]).median()),
                             "epi": float((r[:, 3] - r[:, 2]).median()),
                             "loop_max": float((r[:, 2] - r[:, 1]).max()),
                             "end_spread": float(r[:, 3].max() - r[:, 3].min()),
                             "loop_median_by_xcc": per_xcc,
                             "loop_spread_in_xcc": {int(x): round(float(
                                 loop[xcc == x].max() - loop[xcc == x].min()), 2)
                                 for x in per_xcc}})
            best = min(rows, key=lambda d: d["span"])
            ref = (torch.rand(1, device=dev))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                torch.matmul(x, w.t(), out=out)
            e0.record()
            for _ in range(20):
                torch.matmul(x, w.t(), out=out)
            e1.record()
            e1.synchronize()
            blas = e0.elapsed_time(e1) / 20 * 1e3
            del ref
            print(json.dumps({"M": M, "N": N, "K": K, "nj": nj, "tiles": tiles,
                              **{k: (round(v, 2) if isinstance(v, float) else v)
                                 for k, v in best.items()},
                              "loop_per_ktile_us": round(best["loop"] / (K // 64), 4),
                              "blas_us": round(blas, 2)}), flush=True)


if __name__ == "__main__":
    main()
