"""Static checks of the ctypes ABI (CPU only).

Every ``_lib.lib().dlbb_*`` call in the package must have an entry in ``_lib._SIGS``: without
``argtypes`` ctypes passes Python ints as 32-bit C ints, silently truncating device pointers
(the kernel then faults on the GPU). Every signature must name a ``DLBB_API`` function of the
HIP sources, and the built library (when present) must export it.
"""

import os
import re
import shutil
import subprocess

import pytest

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "distributed_llm_backend_benchmark_amd")


def _sigs():
    from distributed_llm_backend_benchmark_amd.ops import _lib

    return set(_lib._SIGS)


def test_every_called_symbol_has_a_signature():
    used = set()
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(".py"):
                with open(os.path.join(root, f)) as fh:
                    used |= set(re.findall(r"lib\(\)\.(dlbb_[a-z0-9_]+)", fh.read()))
    assert used, "no library calls found"
    missing = sorted(used - _sigs())
    assert not missing, f"called without a ctypes signature: {missing}"


def test_every_signature_is_a_c_api_function():
    api = set()
    csrc = os.path.join(PKG, "csrc")
    for f in os.listdir(csrc):
        if f.endswith(".hip"):
            with open(os.path.join(csrc, f)) as fh:
                api |= set(re.findall(r"DLBB_API\s+[\w\s\*]+?\b(dlbb_[a-z0-9_]+)\s*\(", fh.read()))
    missing = sorted(_sigs() - api)
    assert not missing, f"signatures without a DLBB_API definition: {missing}"


@pytest.mark.skipif(shutil.which("nm") is None, reason="needs nm")
def test_built_library_exports_every_signature():
    from distributed_llm_backend_benchmark_amd.ops.build import LIB_PATH

    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r"\b(dlbb_[a-z0-9_]+)\b", out))
    missing = sorted(_sigs() - exported)
    assert not missing, f"not exported by {LIB_PATH}: {missing}"


def test_signature_argument_counts_match_the_c_api():
    """argtypes must have exactly as many entries as the C function has parameters (a missing
    one shifts every later argument — e.g. the stream — into the wrong register)."""
    from distributed_llm_backend_benchmark_amd.ops import _lib

    csrc = os.path.join(PKG, "csrc")
    nargs = {}
    for f in os.listdir(csrc):
        if f.endswith(".hip"):
            with open(os.path.join(csrc, f)) as fh:
                src = fh.read()
            for m in re.finditer(r"DLBB_API\s+[\w\s\*]+?\b(dlbb_[a-z0-9_]+)\s*\(([^)]*)\)", src):
                params = m.group(2).strip()
                nargs[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    assert len(nargs) > 30, f"parsed only {len(nargs)} C API functions"
    bad = {name: (len(args), nargs.get(name)) for name, (_, args) in _lib._SIGS.items()
           if nargs.get(name) is not None and len(args) != nargs[name]}
    assert not bad, f"argtypes count != C parameter count (argtypes, C): {bad}"


def test_build_id_detects_source_change(tmp_path, monkeypatch):
    """The library's dlbb_build_id() must equal the hash of csrc/ on disk; editing any source
    makes a previously built library refuse to load."""
    import shutil as _sh

    from distributed_llm_backend_benchmark_amd.ops import _lib, build

    csrc = tmp_path / "csrc"
    _sh.copytree(build.CSRC, csrc)
    monkeypatch.setattr(build, "CSRC", str(csrc))
    before = build.source_id()
    hip = csrc / "reduce.hip"
    hip.write_text(hip.read_text() + "\n// touched\n")
    after = build.source_id()
    assert before != after

    def fake_lib(bid):
        class L:
            pass
        lib = L()
        lib.dlbb_build_id = lambda: bid.encode()
        return lib

    assert _lib.check_build_id(fake_lib(after), after) == after
    with pytest.raises(_lib.KernelError, match="built from other sources"):
        _lib.check_build_id(fake_lib(before), after)


def test_built_library_matches_tree():
    from distributed_llm_backend_benchmark_amd.ops import _lib, build

    if not os.path.exists(build.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.lib()            # raises if stale
    assert _lib.check_build_id(lib, build.source_id()) == build.source_id()
