"""Tracing: roctx ranges for rocprofv3 and an optional torch.profiler session.

The reference has no tracing in code — only backend debug logging through env vars
(``CCL_LOG_LEVEL=debug`` ``collectives/3d/launch_dsccl.sh:34``, ``I_MPI_DEBUG=10``
``collectives/3d/launch_mpiccl.sh:12``). Here:

* :func:`range` / :func:`mark` emit roctx ranges (``librocprofiler-sdk-roctx``) that
  ``rocprofv3 --marker-trace`` records next to the kernel trace, so every timed collective
  config, training-step phase and TP forward is attributable in the timeline. Disabled by
  default (zero cost: a no-op context manager); enable with ``DLBB_TRACE=1`` or
  :func:`enable`. The roctx library is loaded lazily and only when enabled.
* :func:`torch_profile` wraps a region in ``torch.profiler`` (CPU + HIP activity) and writes
  one Chrome trace per rank.
* RCCL's own logging passes through the environment (``NCCL_DEBUG=INFO``,
  ``NCCL_DEBUG_SUBSYS``, ``RCCL_LOG_LEVEL``) — the CLIs' ``--env KEY=VAL`` sets them before
  the process group starts; ``HIP_LAUNCH_BLOCKING=1`` serialises every launch for debugging.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Iterator, Optional

_enabled = os.environ.get("DLBB_TRACE", "0") not in ("", "0", "false", "False")
_lib: Optional[ctypes.CDLL] = None
_lib_failed = False

_ROCTX_CANDIDATES = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                     "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4",
                     "/opt/rocm/lib/libroctx64.so.4")


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = bool(on)


def enabled() -> bool:
    return _enabled


def _roctx() -> Optional[ctypes.CDLL]:
    global _lib, _lib_failed
    if _lib is not None or _lib_failed:
        return _lib
    for name in _ROCTX_CANDIDATES:
        try:
            lib = ctypes.CDLL(name)
        except OSError:
            continue
        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        lib.roctxRangePushA.restype = ctypes.c_int
        lib.roctxRangePop.argtypes = []
        lib.roctxRangePop.restype = ctypes.c_int
        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
        lib.roctxMarkA.restype = None
        _lib = lib
        return lib
    _lib_failed = True
    return None


@contextlib.contextmanager
def range(name: str) -> Iterator[None]:  # noqa: A001 - mirrors roctx naming
    """roctx push/pop around the block when tracing is enabled (no-op otherwise)."""
    lib = _roctx() if _enabled else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


def available() -> bool:
    """True if a roctx library can be loaded on this machine."""
    return _roctx() is not None


@contextlib.contextmanager
def torch_profile(out_dir: Optional[str], rank: int = 0) -> Iterator[None]:
    """Profile the block with torch.profiler and export ``<out_dir>/trace_rank<r>.json``.
    ``out_dir=None`` disables it."""
    if not out_dir:
        yield
        return
    import torch
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    os.makedirs(out_dir, exist_ok=True)
    with profile(activities=acts, record_shapes=False) as prof:
        yield
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    prof.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))
