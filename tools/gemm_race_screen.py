"""Race screen for a sync-structure change of the ping-pong GEMMs (CDNA guide: a new
phase/vmcnt placement is a new template — screen it over many runs at several shapes).

Every GEMM here is deterministic (no atomics, fixed reduction order), so each repeat must be
BITWISE equal to the first result; the first result is also checked against an fp32 reference.
NT forward (plain and balanced DMA issue) and NN dgrad (plain and balanced), ragged and
aligned shapes, short and long K, in ONE process. Prints one JSON line per (kind, mode, shape)
and exits non-zero on any mismatch.

    python tools/gemm_race_screen.py [--repeats 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import gemm  # noqa: E402

NT_SHAPES = [(4096, 4096, 4096), (16384, 3072, 768), (4104, 2368, 2048), (2048, 50304, 768),
             (4096, 4096, 16384)]
NN_SHAPES = [(16384, 768, 3072), (16384, 3072, 768), (4104, 1024, 4096), (2048, 768, 50304)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=30)
    args = ap.parse_args()
    bad = 0
    os.environ["DLBB_GEMM"] = "mfma"
    gemm.set_tile(256)
    for kind, shapes in (("nt", NT_SHAPES), ("nn", NN_SHAPES)):
        for bal in (0, 1):
            gemm.set_bal(bal)
            for M, N, K in shapes:
                g = torch.Generator(device="cuda").manual_seed(M + N + K)
                a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                if kind == "nt":
                    b = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    run = lambda: gemm.linear(a, b)  # noqa: E731
                    ref = a.float() @ b.float().t()
                else:
                    b = (torch.rand(K, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                    run = lambda: gemm._dgrad_hip(a, b, out).clone()  # noqa: E731
                    ref = a.float() @ b.float()
                first = run()
                torch.cuda.synchronize()
                err = float((first.float() - ref).abs().max() / ref.abs().max())
                mism = 0
                for _ in range(args.repeats):
                    if not torch.equal(run(), first):
                        mism += 1
                ok = mism == 0 and err < 1e-2
                bad += 0 if ok else 1
                print(json.dumps({"kind": kind, "bal": bal, "M": M, "N": N, "K": K,
                                  "repeats": args.repeats, "mismatches": mism,
                                  "rel_err_vs_fp32": round(err, 5), "ok": ok}), flush=True)
    gemm.set_bal(2)
    gemm.set_tile(0)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
