"""ISA guard for the inline-asm transposed LDS reads (``ds_read_tr16`` in csrc/common.h).

Why the asm form exists: ``__builtin_amdgcn_ds_read_tr16_b64`` carries an LDS memory operand
that the compiler's wait-count pass cannot tell apart from the LDS-DMA (``global_load_lds`` /
``buffer_load ... lds``) still in flight into the OTHER buffer of a double / triple buffered
loop, so it puts ``s_waitcnt vmcnt(0)`` in front of the first such read of every iteration —
draining the prefetch the loop was built to overlap (NN / TN ping-pong GEMMs, the weight-gradient
kernel, all three attention kernels; found in round 5 by reading the ISA). The asm read is
invisible to that pass, so the compiler also never waits for its RESULT: the kernels wait
``lgkmcnt(0)`` themselves before any use. This tool checks that on the compiled code.

Check, per kernel, over the device assembly in program order: after any LDS read written as
inline asm (``ds_read_tr16``, ``ds_read_b128_asm``), its destination registers are PENDING until an ``s_waitcnt`` with ``lgkmcnt(0)`` (counted
``lgkmcnt(N)`` waits do not clear: the compiler cannot have counted the asm reads). Any other
instruction that reads or writes a pending register is a violation (a use of data that may not
have landed, or a write the late LDS return would overwrite). Also reports, per kernel, every
compiler-generated ``s_waitcnt vmcnt(0)`` directly in front of an LDS read (the pattern the asm
form removes).

Usage: ``python tools/isa_check.py [csrc/*.hip ...]`` (default: every csrc source that contains
a transposed read); exit status 1 on any violation.
"""

from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile
from typing import Dict, List, Set, Tuple

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "distributed_llm_backend_benchmark_amd", "csrc")
_REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(text: str) -> Set[Tuple[str, int]]:
    out = set()
    for m in _REG.finditer(text):
        if m.group(1):
            out.update((m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def device_asm(src: str) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "--cuda-device-only", "-S", "-o", out, src]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        with open(out) as f:
            return f.read()


def check_asm(text: str) -> Dict[str, Dict]:
    """{kernel: {"tr_reads": n, "violations": [...], "vmcnt0_before_lds_read": n}}"""
    res: Dict[str, Dict] = {}
    kern = None
    pending: Set[Tuple[str, int]] = set()
    in_asm = False
    lines = text.split("\n")
    for i, line in enumerate(lines):
        m = re.match(r"^(_Z\S+|[A-Za-z_]\w*):\s", line + " ")
        if m and not line.startswith(".") and not line.startswith("\t"):
            if m.group(1).startswith("_Z") or "@" in line:
                kern = m.group(1)
                res.setdefault(kern, {"tr_reads": 0, "violations": [],
                                      "vmcnt0_before_lds_read": 0})
                pending = set()
            continue
        if kern is None:
            continue
        s = line.strip()
        if ";;#ASMSTART" in s:
            in_asm = True
            continue
        if ";;#ASMEND" in s:
            in_asm = False
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        s = s.split(";")[0].strip()
        op = s.split()[0] if s else ""
        if op == "s_endpgm":
            pending = set()
            continue
        if op == "s_waitcnt":
            if "lgkmcnt(0)" in s:
                pending = set()
            if not in_asm and re.search(r"vmcnt\(0\)", s):
                for j in range(i + 1, min(i + 4, len(lines))):
                    t = lines[j].strip()
                    if t.startswith("ds_read"):
                        res[kern]["vmcnt0_before_lds_read"] += 1
                        break
            continue
        if op.startswith("ds_read") and in_asm:   # builtin reads: the compiler counts them
            parts = s[len(op):].split(",")
            dst = regs(parts[0])
            src = regs(",".join(parts[1:]))
            bad = (dst | src) & pending
            if bad:
                res[kern]["violations"].append((i + 1, s, sorted(bad)))
            pending |= dst
            res[kern]["tr_reads"] += 1
            continue
        if pending:
            used = regs(s[len(op):])
            bad = used & pending
            if bad:
                res[kern]["violations"].append((i + 1, s, sorted(bad)))
    return res


def default_sources() -> List[str]:
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hip"):
            p = os.path.join(CSRC, f)
            with open(p) as fh:
                if "ds_read_tr16" in fh.read():
                    out.append(p)
    return out


def main(argv=None) -> int:
    srcs = (argv if argv else None) or default_sources()
    bad = 0
    for src in srcs:
        rep = check_asm(device_asm(src))
        for k, r in rep.items():
            if not r["tr_reads"] and not r["vmcnt0_before_lds_read"]:
                continue
            print(f"{os.path.basename(src)} {k[:80]}: tr_reads={r['tr_reads']} "
                  f"vmcnt0_before_lds_read={r['vmcnt0_before_lds_read']} "
                  f"violations={len(r['violations'])}")
            for v in r["violations"][:5]:
                print(f"    line {v[0]}: {v[1]}  regs {v[2][:6]}")
            bad += len(r["violations"])
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
