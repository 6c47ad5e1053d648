"""Side streams that really run beside the compute stream.

A HIP stream is served by one of the process's hardware queues (``GPU_MAX_HW_QUEUES``, 4 on
this pool). More streams than queues share them, and two streams on ONE hardware queue execute
in order: a "side" stream that landed on the compute stream's queue silently serialises
everything it was meant to overlap. ``torch.cuda.Stream()`` hands out pool streams round-robin,
so whether a new side stream collides depends on how many streams the process (RCCL included)
created before — measured on MI355X (``profiles/r03_tp/overlap_probe``, ``profiles/r03_overlap``):

* the overlapped TP forward: 17.6 ms vs 28.6 ms depending only on how the RCCL communicator was
  initialised before the comm stream was created (no overlap at all in the second case);
* the DDP tail runs: one trainer in four stalled its backward behind the comm stream (+2.1 ms at
  100 GB/s), a different one after changing the communicator init — the stall moved with the
  stream order, not with the configuration.

:func:`concurrent_stream` therefore PROBES candidates: a 1-workgroup spin kernel (~100 us) on
the reference (compute) stream and one on the candidate, started together; if the pair takes
about one spin, the candidate runs concurrently. It also has to run beside every side stream
handed out before on that device (DDP's weight-gradient and comm streams must not share a queue
either). The verified stream is cached per (device, role, priority).
"""

from __future__ import annotations

import warnings
from typing import Dict, Optional, Tuple

import torch

_CACHE: Dict[Tuple[int, str, int], "torch.cuda.Stream"] = {}
# every candidate stream probed, in order: (role, hipStream_t handle, ran beside ref, handed out)
# — result JSONs carry it so a rocprofv3 kernel trace's Stream_Id / Queue_Id columns can be
# matched to roles
LOG: list = []
_PROBE_NS = 100_000
_TRIES = 12


def _pair_ms(a, b, ns: int, device) -> float:
    """Event time around a spin on ``a`` and a spin on ``b`` started together (``b`` None: the
    spin on ``a`` alone)."""
    from ..ops.elementwise import spin_ns

    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    e0.record(a)
    if b is not None:
        b.wait_event(e0)
    with torch.cuda.stream(a):
        spin_ns(ns, 1, device)
    if b is not None:
        with torch.cuda.stream(b):
            spin_ns(ns, 1, device)
        a.wait_stream(b)
    e1.record(a)
    e1.synchronize()
    return e0.elapsed_time(e1)


_BASE: Dict[Tuple[int, int], Tuple[float, float]] = {}


def _baseline(a, device, ns: int) -> Tuple[float, float]:
    """(one spin, two spins in order on ONE stream) on this device, measured the same way as a
    probe pair — the probe's threshold sits between them, so a profiler's per-dispatch overhead
    (rocprofv3 kernel tracing adds 30-90 us to a dispatch on a fresh queue) moves both ends
    instead of turning every candidate into a false "serialised" (profiles/r06_queues)."""
    key = (device.index if device.index is not None else torch.cuda.current_device(), ns)
    if key not in _BASE:
        one = min(_pair_ms(a, None, ns, device) for _ in range(3))
        two = min(_pair_ms(a, a, ns, device) for _ in range(3))
        _BASE[key] = (one, two)
    return _BASE[key]


def runs_concurrently(a, b, device=None, ns: int = _PROBE_NS) -> bool:
    """True if kernels on streams ``a`` and ``b`` overlap in time: the best of two probe pairs
    finishes closer to one spin than to two spins in order (both measured on this device)."""
    dev = device or torch.device("cuda", torch.cuda.current_device())
    one, two = _baseline(a, dev, ns)
    t = min(_pair_ms(a, b, ns, dev) for _ in range(2))
    return t < one + 0.5 * max(two - one, 0.5 * ns * 1e-6)


def concurrent_stream(device, role: str, priority: int = 0,
                      ref: Optional["torch.cuda.Stream"] = None) -> "torch.cuda.Stream":
    """A stream for ``role`` on ``device`` verified to run beside ``ref`` (default: the current
    stream) and beside every side stream already handed out on that device. With more side
    roles than free hardware queues no candidate can satisfy both; it then settles for a stream
    that still runs beside ``ref`` (sharing a queue with another side role: those two roles
    serialise with each other, never with the compute stream), with a warning; only if none of
    ``_TRIES`` pool streams runs beside ``ref`` does it return a serialising one."""
    dev = torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), role, int(priority))
    if key in _CACHE:
        return _CACHE[key]
    ref = ref or torch.cuda.current_stream(dev)
    others = [s for k, s in _CACHE.items() if k[0] == key[0]]
    cand, beside_ref = None, None
    for _ in range(_TRIES):
        cand = torch.cuda.Stream(dev, priority=priority)
        if cand == ref or any(cand == o for o in others):
            continue
        ok = runs_concurrently(ref, cand, dev)
        LOG.append({"role": role, "stream": hex(cand.cuda_stream), "beside_ref": ok,
                    "ref": hex(ref.cuda_stream)})
        if ok:
            if all(runs_concurrently(o, cand, dev) for o in others):
                break
            beside_ref = beside_ref or cand
    else:
        if beside_ref is not None:
            warnings.warn(f"side stream for {role!r} shares a hardware queue with another side "
                          "role (more side roles than free queues); it still overlaps the "
                          "compute stream", RuntimeWarning, stacklevel=2)
            cand = beside_ref
        else:
            warnings.warn(f"no pool stream ran concurrently with the compute stream for "
                          f"{role!r}; overlap on this device will serialise", RuntimeWarning,
                          stacklevel=2)
    _CACHE[key] = cand
    return cand


_GROUPS: Dict[Tuple[int, str, int], list] = {}


def concurrent_group(device, n: int, role: str) -> list:
    """``n`` streams that all run concurrently with each other (not necessarily with the
    current stream): e.g. the W per-rank launches of the virtual-rank harness, whose spinning
    kernels wait for each other — two of them on one hardware queue would serialise until the
    kernels' wall-clock bound. Cached per (device, role, n); with fewer than ``n`` distinct
    queues reachable it returns the best effort (warning)."""
    dev = torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), role, int(n))
    if key in _GROUPS:
        return _GROUPS[key]
    picked: list = []
    for _ in range(_TRIES + 4 * n):
        if len(picked) == n:
            break
        cand = torch.cuda.Stream(dev)
        if any(cand == p for p in picked):
            continue
        if all(runs_concurrently(p, cand, dev) for p in picked):
            picked.append(cand)
    if len(picked) < n:
        warnings.warn(f"only {len(picked)} of {n} mutually concurrent streams found for "
                      f"{role!r}", RuntimeWarning, stacklevel=2)
        while len(picked) < n:
            picked.append(torch.cuda.Stream(dev))
    _GROUPS[key] = picked
    return picked


def reset() -> None:
    """Forget the handed-out streams and probe baselines (tests)."""
    _CACHE.clear()
    _GROUPS.clear()
    _BASE.clear()


# A side stream is ordered after the compute stream by one event record + wait through
# csrc/streams.hip dlbb_stream_fork with a device-scope release (mode 2). GPT-2 step, three
# interleaved reps (profiles/r05_step/SUMMARY.md §7): torch's Stream.wait_stream (default HIP
# event: system-scope fence) 17.89-17.98 ms and one 19.53 ms run (compute-stream dispatch stalled
# ~58 us after every forked-from kernel — the pattern rocprofv3 shows for system-fenced events,
# never for device-scope ones), device-scope 17.86-17.88.
_FORK_MODE = 2


def fork(to: "torch.cuda.Stream", frm: Optional["torch.cuda.Stream"] = None) -> None:
    """``to.wait_stream(frm)`` (default: the current stream) through an event without the
    system-scope fence (cache writeback + invalidate) a default HIP event record performs; two
    streams of one device need only the device-scope ordering every kernel dispatch already
    releases (``profiles/r05_step/SUMMARY.md`` §7)."""
    frm = frm if frm is not None else torch.cuda.current_stream(to.device)
    if to.device.type != "cuda":
        to.wait_stream(frm)
        return
    from ..ops import _lib

    # the event ring is per device (csrc/streams.hip picks it by the current device): make it
    # the streams' device, whatever device is current
    with torch.cuda.device(to.device):
        rc = _lib.lib().dlbb_stream_fork(frm.cuda_stream, to.cuda_stream, _FORK_MODE)
    if rc != 0:
        raise RuntimeError(f"dlbb_stream_fork failed (hip error {rc})")
