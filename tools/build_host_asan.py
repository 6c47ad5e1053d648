"""Build tests/native/host_checks.cpp against the kernel library with AddressSanitizer,
LeakSanitizer and UBSan on the HOST code (``-Xarch_host -fsanitize=...``; device code is not
instrumented). Output: ``build/asan/host_checks``. Incremental like ops/build.py."""

from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_llm_backend_benchmark_amd.ops.build import ARCH, CSRC, ROCM, hipcc, sources  # noqa

OUT = os.path.join(REPO, "build", "asan")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-omit-frame-pointer"]
FLAGS = ["-O1", "-g", "-std=c++17", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *SAN]


def _newer(dst, *srcs):
    return os.path.exists(dst) and all(os.path.getmtime(dst) >= os.path.getmtime(s) for s in srcs)


def _compile(src):
    obj = os.path.join(OUT, os.path.basename(src).rsplit(".", 1)[0] + ".o")
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if _newer(obj, *deps):
        return obj
    r = subprocess.run([hipcc(), *FLAGS, "-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"asan compile failed for {src}:\n{r.stderr}")
    return obj


def build() -> str:
    os.makedirs(OUT, exist_ok=True)
    srcs = sources() + [os.path.join(REPO, "tests", "native", "host_checks.cpp")]
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(_compile, srcs))
    exe = os.path.join(OUT, "host_checks")
    if not _newer(exe, *objs):
        r = subprocess.run([hipcc(), f"--offload-arch={ARCH}", *SAN, "-o", exe, *objs,
                            f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"asan link failed:\n{r.stderr}")
    return exe


if __name__ == "__main__":
    print(build())
