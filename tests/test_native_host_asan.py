"""Host-side AddressSanitizer / LeakSanitizer / UBSan run of the kernel library's C ABI
(tests/native/host_checks.cpp, built by tools/build_host_asan.py with -Xarch_host
-fsanitize=...). Without a GPU every entry point must fail cleanly and leak nothing; on the GPU
box the IPC all-reduce state is created and destroyed for real."""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(expect_devices):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from build_host_asan import build

    exe = build()
    supp = os.path.join(REPO, "tests", "native", "lsan.supp")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:"
                                        "halt_on_error=1",
               LSAN_OPTIONS=f"suppressions={supp}:print_suppressions=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=150, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "ERROR: LeakSanitizer" not in out, out[-4000:]
    assert "runtime error" not in out, out[-4000:]          # UBSan
    line = [l for l in r.stdout.splitlines() if l.startswith("host checks")][-1]
    assert "failures=0" in line
    if expect_devices:
        assert "devices=0" not in line, line


def test_host_asan_no_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("device visible: covered by the gpu variant")
    _run(expect_devices=False)


@pytest.mark.gpu
def test_host_asan_with_device():
    _run(expect_devices=True)
