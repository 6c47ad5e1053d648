"""Per-kernel register / scratch / occupancy table of every csrc/*.hip kernel for gfx950, from
the compiler's own resource report (``-Rpass-analysis=kernel-resource-usage``, device-only
compile, CPU only). A kernel that keeps an array in private memory (``ScratchSize`` > 0, e.g. a
register array indexed dynamically after an epilogue grew past the unroll threshold) runs its
hot loop through scratch: ``tests/test_kernel_resources.py`` fails on that.

usage: python tools/kernel_resources.py [--json]
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import re
import subprocess
import sys
from typing import Dict, List

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_backend_benchmark_amd.ops import build  # noqa: E402

_FIELDS = {"VGPRs": "vgprs", "AGPRs": "agprs", "ScratchSize [bytes/lane]": "scratch",
           "Occupancy [waves/SIMD]": "occupancy", "VGPRs Spill": "vgpr_spill",
           "SGPRs Spill": "sgpr_spill", "LDS Size [bytes/block]": "lds_static"}


def _report(src: str) -> List[Dict]:
    cmd = [build.hipcc(), "-O3", "-std=c++17", f"--offload-arch={build.ARCH}",
           "--cuda-device-only", "-c", src, "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-2000:]}")
    out: List[Dict] = []
    cur = None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"file": os.path.basename(src), "kernel": m.group(1)}
            out.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z][^:]*): (\d+)", line)
        if m and cur is not None and m.group(1) in _FIELDS:
            cur[_FIELDS[m.group(1)]] = int(m.group(2))
    return out


def collect() -> List[Dict]:
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        rows = [r for rs in ex.map(_report, build.sources()) for r in rs]
    return sorted(rows, key=lambda r: (r["file"], r["kernel"]))


def main() -> int:
    rows = collect()
    if "--json" in sys.argv:
        for r in rows:
            print(json.dumps(r))
        return 0
    print(f"{'file':22s} {'vgpr':>4s} {'agpr':>4s} {'scr':>4s} {'occ':>3s}  kernel")
    for r in rows:
        print(f"{r['file']:22s} {r.get('vgprs', 0):4d} {r.get('agprs', 0):4d} "
              f"{r.get('scratch', 0):4d} {r.get('occupancy', 0):3d}  {r['kernel'][:90]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
