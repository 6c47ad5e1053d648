"""CPU guard on the compiled gfx950 code (hipcc cross-compiles here): every inline-asm LDS read
(csrc/common.h ds_read_tr16 / ds_read_b128_asm) is waited for (lgkmcnt(0)) before any
instruction touches its registers, and no kernel has a compiler-inserted vmcnt(0) drain in
front of an LDS read (tools/isa_check.py)."""
import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

pytestmark = pytest.mark.skipif(not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")),
                                reason="needs hipcc")


@pytest.mark.parametrize("src", ["attention.hip", "gemm_tn.hip", "gemm.hip"])
def test_asm_lds_reads_are_waited_for(src):
    import isa_check

    path = os.path.join(isa_check.CSRC, src)
    rep = isa_check.check_asm(isa_check.device_asm(path))
    reads = sum(r["tr_reads"] for r in rep.values())
    assert reads > 0, "no asm LDS reads found: the checker is not looking at the right code"
    bad = {k: r["violations"][:3] for k, r in rep.items() if r["violations"]}
    assert not bad, bad
    drains = {k: r["vmcnt0_before_lds_read"] for k, r in rep.items()
              if r["vmcnt0_before_lds_read"] and not any(a in k for a in ALLOWED_DRAINS)}
    assert not drains, drains


# kernels that keep the builtin transposed read on purpose (measured faster, see the source)
ALLOWED_DRAINS = ("attn_fwd_kernel",)


def test_checker_flags_an_early_use():
    import isa_check

    asm = """
_Z1kv:                                  ; @_Z1kv
\t;;#ASMSTART
\tds_read_b64_tr_b16 v[2:3], v1 offset:0
\t;;#ASMEND
\tv_add_u32_e32 v4, v2, v5
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(0)
\t;;#ASMEND
\tv_add_u32_e32 v6, v3, v5
\ts_endpgm
"""
    rep = isa_check.check_asm(asm)["_Z1kv"]
    assert rep["tr_reads"] == 1
    assert len(rep["violations"]) == 1 and "v4" in rep["violations"][0][1]


def test_compiler_drains_lds_dma_before_builtin_transposed_read():
    """The reason for the asm reads, pinned: with the builtin the compiler waits vmcnt(0) for
    the other buffer's LDS-DMA before the read; a plain LDS load and the asm read do not wait
    (tools/diag/lds_dma_wait.hip). If a future compiler stops doing it, this test says so."""
    import re

    import isa_check

    asm = isa_check.device_asm(os.path.join(REPO, "tools", "diag", "lds_dma_wait.hip"))
    funcs = {}
    cur = None
    for line in asm.split("\n"):
        m = re.match(r"^(k_\w+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur:
            funcs[cur].append(line.strip())

    def vmcnt0_before_lds_read(lines):
        for i, s in enumerate(lines):
            if s.startswith("ds_read"):
                prev = [x for x in lines[max(0, i - 3):i] if x.startswith("s_waitcnt")]
                return any("vmcnt(0)" in x for x in prev)
        raise AssertionError("no LDS read found")

    assert vmcnt0_before_lds_read(funcs["k_builtin"])
    assert not vmcnt0_before_lds_read(funcs["k_plain"])
    assert not vmcnt0_before_lds_read(funcs["k_asm"])
