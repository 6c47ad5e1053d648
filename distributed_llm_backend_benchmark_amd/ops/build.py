"""Build the gfx950 HIP kernel library in-tree.

``python -m distributed_llm_backend_benchmark_amd.ops.build`` compiles every ``csrc/*.hip``
with ``hipcc --offload-arch=gfx950`` into objects under ``build/`` and links
``<package>/_dlbb_hip.so`` (a plain C-ABI shared library, loaded with ctypes by
:mod:`._lib`). No torch headers, no hipify: the sources are HIP/CDNA4 code written for gfx950.
Incremental by CONTENT: an object is rebuilt when the hash of its source + headers + flags
differs from the stamp next to it (never by timestamps, which tar / copies do not preserve
reliably). The library carries ``dlbb_build_id()`` = hash of every ``csrc`` source and header
and the flags (:func:`source_id`); :mod:`._lib` refuses to load a library whose id does not
match the sources on disk, so a tested binary is always the committed ``csrc/``.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from typing import List

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
REPO = os.path.dirname(PKG_DIR)
BUILD = os.path.join(REPO, "build", "hip")
LIB_NAME = "_dlbb_hip.so"
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)
ARCH = os.environ.get("DLBB_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-function", "-munsafe-fp-atomics"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError("hipcc not found (need ROCm: /opt/rocm/bin/hipcc)")


def sources() -> List[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _digest(paths: List[str]) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(CFLAGS).encode())
    return h.hexdigest()[:16]


def _headers() -> List[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))


def source_id() -> str:
    """Hash of every csrc source and header and the compile flags: the id the library must
    carry (``dlbb_build_id``)."""
    return _digest(sources() + _headers())


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


def _compile(src: str, verbose: bool) -> str:
    obj = os.path.join(BUILD, os.path.basename(src)[:-4] + ".o")
    stamp = _digest([src] + _headers())
    if os.path.exists(obj) and _read(obj + ".sha") == stamp:
        return obj
    cmd = [hipcc(), *CFLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    with open(obj + ".sha", "w") as f:
        f.write(stamp)
    return obj


def _build_id_object(bid: str) -> str:
    """A host-only object exporting ``const char* dlbb_build_id(void)``."""
    src = os.path.join(BUILD, "build_id.c")
    obj = os.path.join(BUILD, "build_id.o")
    with open(src, "w") as f:
        f.write('__attribute__((visibility("default"))) const char* dlbb_build_id(void) '
                f'{{ return "{bid}"; }}\n')
    cc = shutil.which("gcc") or shutil.which("cc") or hipcc()
    r = subprocess.run([cc, "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build id object failed:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False, jobs: int = 0) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    if force:
        for s in srcs:
            o = os.path.join(BUILD, os.path.basename(s)[:-4] + ".o")
            if os.path.exists(o):
                os.remove(o)
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    bid = source_id()
    if force or not os.path.exists(LIB_PATH) or _read(LIB_PATH + ".buildid") != bid:
        tmp = LIB_PATH + f".tmp{os.getpid()}"
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs,
               _build_id_object(bid), f"-L{ROCM}/lib", "-lrccl"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB_PATH)
        with open(LIB_PATH + ".buildid", "w") as f:
            f.write(bid)
    return LIB_PATH


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    args = ap.parse_args(argv)
    path = build(force=args.force, verbose=args.verbose, jobs=args.jobs)
    print(f"built {path}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
