"""Compile-time resource guard for every gfx950 kernel (CPU only: hipcc's own report).

No kernel may keep data in scratch (private memory) or spill VGPRs — a register array that
becomes dynamically indexed (e.g. once an epilogue grows past the unroll threshold) silently
moves the whole accumulator tile to scratch and costs far more than the change that caused it.
(Round 5's one exception, the persistent deep-pipeline 256^2 GEMM, was removed in round 6.)
"""

import os
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

# Measured exceptions. The dK/dV attention kernel at 3 workgroups per CU spills 4 VGPRs (20 B of
# scratch per lane). Its 768-workgroup causal-paired grid then fits one round instead of 1.5.
# At the GPT-2 shape the whole backward runs 142-146 us against 156-158 us without the spill
# (profiles/r06_kernels/attn_bwd_dkdv_3wg_ab.jsonl).
ALLOWED_SCRATCH: dict = {"_ZN4dlbb24attn_bwd_dkdv_d64_kernelILb0EEEvNS_11AttnBwdArgsE": 20}


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_no_scratch_or_spills_in_kernels():
    import kernel_resources

    rows = kernel_resources.collect()
    assert len(rows) > 50, "resource report parsed too few kernels"
    names = {r["kernel"] for r in rows}
    for must in ("gemm_bf16_nt_256_pingpong3", "wgrad_kernel", "attn_bwd_dkdv_d64_kernel",
                 "xent_fused2_kernel", "car_rs_kernel", "adamw_kernel"):
        assert any(must in n for n in names), f"no kernel matching {must!r} in the report"
    bad = []
    for r in rows:
        limit = ALLOWED_SCRATCH.get(r["kernel"], 0)
        if r.get("scratch", 0) > limit or (limit == 0 and r.get("vgpr_spill", 0) > 0):
            bad.append((r["file"], r["kernel"], r.get("scratch"), r.get("vgpr_spill")))
    assert not bad, f"kernels using scratch / spilling: {bad}"
