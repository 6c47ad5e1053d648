"""IPC one-shot / two-shot xGMI all-reduce (``csrc/custom_allreduce.hip``).

The oneCCL algorithm sweep of the reference (``CCL_ALLREDUCE`` ∈ direct/ring/2d/...,
``collectives/3d/launch_dsccl.sh:46-47``) maps here to three all-reduce implementations on one
node: RCCL (ring/tree, default), ``oneshot`` (every rank reads all peers' full buffers over its
7 dedicated xGMI links — the "direct" analogue, lowest latency) and ``twoshot`` (direct
reduce-scatter + direct all-gather — the "2d"/rabenseifner analogue, all links busy).
``register(t)`` IPC-maps a user tensor on every rank once; ``all_reduce_registered`` then runs
the two-shot in place on it (no copy-in, no staging buffer: the bandwidth path for large,
long-lived buffers such as gradient buckets or a benchmark's message). The same registration
serves the direct one-hop ``all_gather_registered`` / ``reduce_scatter_registered`` /
``all_to_all_registered`` kernels: each GPU pulls its peers' data over its 7 xGMI links at once.

Setup: each rank allocates its IPC regions, the 192-byte handles and device ordinals are
exchanged once through the process group (``all_gather_object``), peers are opened with
``hipIpcOpenMemHandle``. ``auto`` selection uses the custom kernel only below a crossover
size and only after a start-up self-test against RCCL passed on every rank.
"""

from __future__ import annotations

import ctypes
import os
import time
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import _lib
from .comm import Comm

ONESHOT, TWOSHOT = 1, 2
DIRECT_AG, DIRECT_A2A, DIRECT_RS = 0, 1, 2

_INSTANCES: Dict[int, "CustomAllReduce"] = {}


# Crossovers. Measured with the single-GPU virtual-rank harness (tools/car_harness.py, one fused
# launch of the production kernels for W ranks; profiles/r02_car_harness/SUMMARY.md, "crossover"):
#   * one-shot vs staged two-shot: equal within noise up to 512 KiB at W = 2 / 4 / 8 (e.g. W=8:
#     13.7 vs 13.7 us at 256 KiB, 13.5 vs 13.7 us at 512 KiB); from 1 MiB two-shot is ahead at
#     W = 8 (16.2 vs 16.6 us, 2 MiB 23.3 vs 23.5 us, 8 MiB 68 vs 83 us). On real xGMI each link
#     carries n bytes per one-shot call but only 2n/W per two-shot call, which moves the
#     crossover further down, never up: ONESHOT_MAX = 256 KiB.
#   * the registered in-place two-shot (no copy-in, no staging) is the fastest form at every
#     size measured (W=8: 10.0 us at 64 KiB, 31 us at 8 MiB vs 68 us staged), so long-lived
#     buffers (DDP buckets, benchmark messages) are registered once and use it.
#   * custom vs RCCL (AUTO_MAX = 8 MiB) cannot be measured on one GPU (RCCL needs one GPU per
#     rank); bench.py times every candidate per size on the driver's multi-GPU node and keeps
#     the fastest validated one, which is what its JSON reports.
ONESHOT_MAX_BYTES = 256 << 10
AUTO_MAX_BYTES = 8 << 20
# Those two constants are only the defaults: at world > 1 the instance re-derives both on the
# node it runs on (:meth:`CustomAllReduce.calibrate`, the analogue of the reference's per-message
# CCL_ALLREDUCE algorithm choice, collectives/3d/launch_dsccl.sh:46-47): RCCL vs one-shot /
# two-shot / registered pull / push timed at CALIB_SIZES, rank-max, agreed by every rank.
CALIB_SIZES = (4 << 10, 64 << 10, 512 << 10, 4 << 20, 16 << 20, 64 << 20)


class CustomAllReduce:
    def __init__(self, comm: Comm, capacity_bytes: int = 64 << 20,
                 oneshot_max_bytes: int = ONESHOT_MAX_BYTES,
                 auto_max_bytes: int = AUTO_MAX_BYTES,
                 nblocks: Optional[int] = None):
        if not comm.is_gpu:
            raise RuntimeError("custom all-reduce needs HIP devices")
        if comm.world_size > 8:
            raise RuntimeError("custom all-reduce supports up to 8 ranks (one node)")
        self.comm = comm
        self.lib = _lib.lib()
        self.h = None
        # Every step that can fail locally is followed by an all-ranks agreement, so one rank's
        # failure (allocation, IPC export/open, peer access) never leaves the others blocked in
        # a collective.
        mine, err = None, None
        try:
            h = ctypes.c_void_p()
            _lib.check(self.lib.dlbb_car_create(comm.rank, comm.world_size, int(capacity_bytes),
                                                ctypes.byref(h)), "car_create")
            self.h = h
            buf = ctypes.create_string_buffer(self.lib.dlbb_car_handle_bytes())
            _lib.check(self.lib.dlbb_car_ipc_handles(self.h, buf), "car_ipc_handles")
            mine = bytes(buf.raw)
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = e
        allh = comm.all_gather_object((mine, torch.cuda.current_device(), repr(err)))
        if any(x[0] is None for x in allh):
            self.close()
            raise RuntimeError(f"custom all-reduce setup failed: {[x[2] for x in allh]}")
        blob = b"".join(x[0] for x in allh)
        devs = (ctypes.c_int * comm.world_size)(*[int(x[1]) for x in allh])
        rc = self.lib.dlbb_car_open(self.h, blob, devs)
        oks = comm.all_gather_object(rc)
        if any(r != 0 for r in oks):
            self.close()
            raise RuntimeError(f"custom all-reduce IPC open failed (hip rc per rank: {oks})")
        self.capacity = int(self.lib.dlbb_car_capacity(self.h))
        self.oneshot_max = oneshot_max_bytes
        self.auto_max = auto_max_bytes
        self.nblocks = nblocks
        self.healthy = False
        self.reg_healthy = False
        self.push_healthy = False
        self.calibration: Optional[dict] = None
        self._regs: Dict[tuple, int] = {}
        self._reg_keep: Dict[int, torch.Tensor] = {}   # rid -> registered tensor (kept alive)
        self._reg_refs: Dict[int, int] = {}            # rid -> register() calls not released
        self._owned: Dict[tuple, Tuple[torch.Tensor, int]] = {}   # (numel, dtype, slot) -> ...

    # ------------------------------------------------------------------ policy
    def supports(self, t: torch.Tensor) -> bool:
        if t.dtype not in (torch.bfloat16, torch.float16, torch.float32) or not t.is_contiguous():
            return False
        nbytes = t.numel() * t.element_size()
        vec = 8 * t.element_size()
        return 0 < nbytes <= self.capacity and nbytes % vec == 0

    def should_use(self, t: torch.Tensor) -> bool:
        return (self.healthy and self.supports(t)
                and t.numel() * t.element_size() <= self.auto_max)

    def algo_for(self, nbytes: int, vec: int) -> int:
        if nbytes <= self.oneshot_max or nbytes % (vec * self.comm.world_size) != 0:
            return ONESHOT
        return TWOSHOT

    def blocks_for(self, nbytes: int, algo: int) -> int:
        if self.nblocks:
            return self.nblocks
        # ~64 KiB of message per workgroup, 1..128 workgroups (256 via nblocks=)
        per = max(1, nbytes // (64 << 10))
        return int(min(128, max(1, per if algo == TWOSHOT else min(per, 32))))

    # ------------------------------------------------------------------ registration
    def register(self, t: torch.Tensor) -> int:
        """Collective: IPC-map tensor ``t`` of every rank (same numel / dtype everywhere) for
        :meth:`all_reduce_registered`. Every local failure is agreed on by all ranks (then
        every rank raises). Registered tensors are kept alive by this object until
        :meth:`deregister`."""
        if (t.dtype not in (torch.bfloat16, torch.float16, torch.float32)
                or not t.is_contiguous() or t.numel() * t.element_size() % 16):
            raise ValueError(f"cannot register {t.numel()} x {t.dtype}")
        key = (t.data_ptr(), t.numel() * t.element_size())
        if key in self._regs:                 # same tensor again: one more reference
            self._reg_refs[self._regs[key]] += 1
            return self._regs[key]
        mine, err = None, None
        try:
            hb = ctypes.create_string_buffer(64)
            off = ctypes.c_int64()
            _lib.check(self.lib.dlbb_car_reg_export(self.h, t.data_ptr(), hb,
                                                    ctypes.byref(off)), "car_reg_export")
            mine = (bytes(hb.raw), int(off.value))
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = e
        allh = self.comm.all_gather_object((mine, repr(err)))
        if any(x[0] is None for x in allh):
            raise RuntimeError(f"custom all-reduce registration failed: {[x[1] for x in allh]}")
        blob = b"".join(x[0][0] for x in allh)
        offs = (ctypes.c_int64 * self.comm.world_size)(*[x[0][1] for x in allh])
        rid = ctypes.c_int(-1)
        rc = self.lib.dlbb_car_reg_open(self.h, t.data_ptr(), key[1], blob, offs,
                                        ctypes.byref(rid))
        oks = self.comm.all_gather_object(rc)
        if any(r != 0 for r in oks):
            raise RuntimeError(f"custom all-reduce registration open failed (hip rc: {oks})")
        self._regs[key] = int(rid.value)
        self._reg_keep[int(rid.value)] = t
        self._reg_refs[int(rid.value)] = 1
        return int(rid.value)

    def deregister(self, rid: int) -> None:
        """Collective: drop one reference to registration ``rid``; at the last one release it on
        every rank — the peer IPC mappings no
        other live registration uses are closed and the tensor is no longer kept alive. Every
        rank first drains its stream and meets the others at a barrier, so no kernel on any rank
        still reads or writes the buffers being unmapped."""
        if rid not in self._reg_keep:
            raise KeyError(f"registration {rid} is not live")
        self._reg_refs[rid] -= 1             # (identical on every rank: same call sequence)
        if self._reg_refs[rid] > 0:
            return
        del self._reg_refs[rid]
        torch.cuda.synchronize(self.comm.device)
        self.comm.barrier()
        rc = self.lib.dlbb_car_reg_close(self.h, int(rid))
        oks = self.comm.all_gather_object(rc)
        t = self._reg_keep.pop(rid)
        self._regs.pop((t.data_ptr(), t.numel() * t.element_size()), None)
        # every rank unmapped before any rank lets its buffer go back to the allocator
        self.comm.barrier()
        if any(r != 0 for r in oks):
            raise RuntimeError(f"custom all-reduce deregistration failed (hip rc: {oks})")

    def registered_buffer(self, numel: int, dtype: torch.dtype,
                          slot: int = 0) -> Tuple[torch.Tensor, int]:
        """Collective on first use of a (numel, dtype): a flat buffer owned by this instance,
        IPC-registered on every rank — a producer (e.g. the row-parallel GEMM) writes straight
        into it and :meth:`all_reduce_registered` reduces it in place. The same buffer comes
        back on later calls (callers must consume it before the next producer writes it);
        ``slot`` keeps separate buffers for producers in flight at once (micro-batches)."""
        key = (int(numel), dtype, int(slot))
        ent = self._owned.get(key)
        if ent is None:
            buf = torch.empty(int(numel), dtype=dtype, device=self.comm.device)
            ent = (buf, self.register(buf))
            self._owned[key] = ent
        return ent

    def reg_counts(self) -> Tuple[int, int]:
        """(live registrations, opened peer IPC mappings) of this rank."""
        live, maps = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.dlbb_car_reg_counts(self.h, ctypes.byref(live), ctypes.byref(maps)),
                   "car_reg_counts")
        return int(live.value), int(maps.value)

    def supports_registered(self, t: torch.Tensor) -> bool:
        if t.dtype not in (torch.bfloat16, torch.float16, torch.float32) or not t.is_contiguous():
            return False
        nbytes = t.numel() * t.element_size()
        return nbytes > 0 and nbytes % (8 * t.element_size() * self.comm.world_size) == 0

    def all_reduce_registered(self, t: torch.Tensor, rid: int, nblocks: Optional[int] = None,
                              push: bool = False) -> torch.Tensor:
        """In-place two-shot on registration ``rid`` (``t`` must be the registered tensor).
        ``push``: remote writes into the peers' staging halves + result pushes instead of
        remote reads (needs ``t`` to fit the staging capacity)."""
        nbytes = t.numel() * t.element_size()
        nb = nblocks or self.nblocks or int(min(256, max(1, nbytes // (256 << 10))))
        fn = self.lib.dlbb_car_allreduce_reg_push if push else self.lib.dlbb_car_allreduce_reg
        _lib.check(fn(self.h, rid, t.numel(), _lib.dt(t), nb, _lib.stream(t.device)),
                   "car_allreduce_reg" + ("_push" if push else ""))
        return t

    def _direct(self, kind: int, t: torch.Tensor, rid: int, out: torch.Tensor, nbytes: int,
                nblocks: Optional[int]) -> torch.Tensor:
        if not out.is_contiguous() or out.dtype != t.dtype:
            raise ValueError("direct collective: out must be contiguous, same dtype as input")
        nb = nblocks or self.nblocks or int(min(256, max(8, nbytes // (256 << 10))))
        _lib.check(self.lib.dlbb_car_direct_reg(self.h, rid, kind, nbytes, _lib.dt(t),
                                                out.data_ptr(), nb, _lib.stream(t.device)),
                   "car_direct_reg")
        return out

    def all_gather_registered(self, t: torch.Tensor, rid: int, out: torch.Tensor,
                              nblocks: Optional[int] = None) -> torch.Tensor:
        """out[p * n : (p + 1) * n] = t of rank p (t registered as ``rid``; out world x n)."""
        if out.numel() != t.numel() * self.comm.world_size:
            raise ValueError("all_gather_registered: out must hold world x input")
        return self._direct(DIRECT_AG, t, rid, out, t.numel() * t.element_size(), nblocks)

    def all_to_all_registered(self, t: torch.Tensor, rid: int, out: torch.Tensor,
                              nblocks: Optional[int] = None) -> torch.Tensor:
        """Equal splits: out chunk p = chunk ``rank`` of rank p's t (t, out: world x c)."""
        W = self.comm.world_size
        if out.numel() != t.numel() or t.numel() % W:
            raise ValueError("all_to_all_registered: in/out of world x chunk elements")
        return self._direct(DIRECT_A2A, t, rid, out, t.numel() // W * t.element_size(), nblocks)

    def all_to_allv_registered(self, t: torch.Tensor, rid: int, out: torch.Tensor, src_off,
                               counts, dst_off, nblocks: Optional[int] = None) -> torch.Tensor:
        """Uneven all-to-all (MoE dispatch) on registration ``rid``: from every peer p,
        ``out[dst_off[p] : + counts[p]] = t_p[src_off[p] : + counts[p]]`` (ELEMENTS, every
        offset / count a multiple of 16 bytes). Collective; t registered with the same size on
        every rank."""
        W = self.comm.world_size
        esz = t.element_size()
        if not out.is_contiguous() or out.dtype != t.dtype or len(counts) != W:
            raise ValueError("all_to_allv_registered: contiguous out of t's dtype, W counts")
        if max(d + c for d, c in zip(dst_off, counts)) > out.numel():
            raise ValueError("all_to_allv_registered: out too small for the receive layout")

        def arr(vals):
            return (ctypes.c_int64 * W)(*[int(v) * esz for v in vals])
        # the grid must be the same on every rank (workgroup b of each rank meets workgroup b of
        # its peers at the flag barriers): size it from the registered input, equal everywhere,
        # never from this rank's own (uneven) receive total
        size = t.numel() * esz
        nb = nblocks or self.nblocks or int(min(256, max(8, size // (256 << 10))))
        _lib.check(self.lib.dlbb_car_alltoallv_reg(self.h, rid, arr(src_off), arr(counts),
                                                   arr(dst_off), out.data_ptr(), nb,
                                                   _lib.stream(t.device)), "car_alltoallv_reg")
        return out

    def reduce_scatter_registered(self, t: torch.Tensor, rid: int, out: torch.Tensor,
                                  nblocks: Optional[int] = None) -> torch.Tensor:
        """out = shard ``rank`` of sum_p t_p (fp32 accumulation; out n / world)."""
        if out.numel() * self.comm.world_size != t.numel():
            raise ValueError("reduce_scatter_registered: out must hold input / world")
        return self._direct(DIRECT_RS, t, rid, out, t.numel() * t.element_size(), nblocks)

    # ------------------------------------------------------------------ ops
    def all_reduce(self, inp: torch.Tensor, out: Optional[torch.Tensor] = None,
                   algo: Optional[int] = None, nblocks: Optional[int] = None) -> torch.Tensor:
        if not self.supports(inp):
            raise ValueError(f"custom all-reduce cannot take {inp.numel()} x {inp.dtype}")
        out = inp if out is None else out
        nbytes = inp.numel() * inp.element_size()
        a = algo or self.algo_for(nbytes, 8 * inp.element_size())
        _lib.check(self.lib.dlbb_car_allreduce(
            self.h, inp.data_ptr(), out.data_ptr(), inp.numel(), _lib.dt(inp), a,
            nblocks or self.blocks_for(nbytes, a), _lib.stream(inp.device)), "car_allreduce")
        return out

    def all_reduce_(self, t: torch.Tensor, algo: Optional[int] = None,
                    nblocks: Optional[int] = None) -> torch.Tensor:
        return self.all_reduce(t, t, algo, nblocks)

    def check_error(self) -> int:
        """This rank's device-side timeout flag (read and cleared; synchronous)."""
        return int(self.lib.dlbb_car_error(self.h))

    def raise_if_error(self) -> None:
        """Collective: if any rank's IPC kernel timed out in a spin wait since the last check
        (its result is partial and the double-buffer reuse guarantee is void), raise on EVERY
        rank. Call outside timed regions: one synchronous 4-byte read + one object all-gather."""
        flags = self.comm.all_gather_object(self.check_error())
        if any(flags):
            bad = [i for i, f in enumerate(flags) if f]
            raise RuntimeError(f"custom all-reduce timed out on ranks {bad}: results since the "
                               "last check are partial; restart the job")

    def self_test(self) -> bool:
        """Compare one-shot and two-shot against RCCL on small/medium messages; all ranks must
        pass for ``healthy``."""
        ok = True
        dev = self.comm.device
        for n in (4096, 1 << 18, 1 << 22):
            if n * 2 > self.capacity:
                continue
            g = torch.Generator(device=dev)
            g.manual_seed(1234 + self.comm.rank)
            x = torch.randn(n, generator=g, device=dev).to(torch.bfloat16)
            ref = x.float().clone()
            if self.comm.world_size > 1:
                dist.all_reduce(ref)
            for algo in (ONESHOT, TWOSHOT):
                for _ in range(2):     # two epochs: both halves of the double buffer
                    try:
                        y = self.all_reduce(x.clone(), algo=algo)
                        torch.cuda.synchronize(dev)
                        good = torch.allclose(y.float(), ref, rtol=2e-2,
                                              atol=5e-2 * self.comm.world_size)
                        ok = ok and good and self.check_error() == 0
                    except Exception:  # noqa: BLE001 - a failed launch is a failed test
                        ok = False
        flags = self.comm.all_gather_object(bool(ok))
        self.healthy = all(flags)
        if not self.healthy and self.comm.rank == 0:
            print(f"[custom all-reduce] self-test failed on ranks "
                  f"{[i for i, f in enumerate(flags) if not f]}: RCCL will be used", flush=True)
        if self.healthy:
            self._self_test_registered()
        return self.healthy

    def _self_test_registered(self) -> None:
        """Registered in-place two-shot, pull and push forms, vs RCCL: six calls alternating the
        forms, each followed by a staged two-shot call on other data, so both staging halves are
        re-read after local writes of the other form. ``reg_healthy`` /
        ``push_healthy`` only if the form passes on every rank. The test buffer is released."""
        dev, W = self.comm.device, self.comm.world_size
        ok = {False: True, True: True}
        rid = None
        try:
            n = 1 << 20
            buf = torch.empty(n, device=dev, dtype=torch.bfloat16)
            rid = self.register(buf)
            for it in range(6):
                push = bool(it % 2)
                g = torch.Generator(device=dev)
                g.manual_seed(777 + 31 * it + self.comm.rank)
                x = torch.randn(n, generator=g, device=dev).to(torch.bfloat16)
                y = torch.randn(n // 4, generator=g, device=dev).to(torch.bfloat16)
                ref, ref_y = x.float().clone(), y.float().clone()
                if W > 1:
                    dist.all_reduce(ref)
                    dist.all_reduce(ref_y)
                buf.copy_(x)
                try:
                    self.all_reduce_registered(buf, rid, push=push)
                    self.all_reduce(y, algo=TWOSHOT)
                    torch.cuda.synchronize(dev)
                    good = bool(torch.allclose(buf.float(), ref, rtol=2e-2, atol=5e-2 * W))
                    good_y = bool(torch.allclose(y.float(), ref_y, rtol=2e-2, atol=5e-2 * W))
                    ok[push] = ok[push] and good and good_y and self.check_error() == 0
                except Exception:  # noqa: BLE001 - a failed launch is a failed test
                    ok[push] = False
        except Exception:  # noqa: BLE001 - a failed registration fails both forms
            ok = {False: False, True: False}
        flags = self.comm.all_gather_object((bool(ok[False]), bool(ok[True]), rid is not None))
        self.reg_healthy = all(f[0] for f in flags)
        self.push_healthy = self.reg_healthy and all(f[1] for f in flags)
        if all(f[2] for f in flags):
            self.deregister(rid)
        if not self.push_healthy and self.comm.rank == 0:
            print("[custom all-reduce] registered-buffer self-test failed (pull/push per rank): "
                  f"{flags}", flush=True)

    # ------------------------------------------------------------------ calibration
    def _time_calls(self, fn, iters: int) -> float:
        """Seconds per call of ``iters`` back-to-back calls on this rank (barrier first, host
        clock around a synchronize on both sides)."""
        for _ in range(2):
            fn()
        torch.cuda.synchronize(self.comm.device)
        self.comm.barrier()
        torch.cuda.synchronize(self.comm.device)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize(self.comm.device)
        return (time.perf_counter() - t0) / iters

    def calibrate(self, sizes=CALIB_SIZES, iters: int = 20) -> dict:
        """Collective: time the process group's all-reduce (RCCL) against the IPC forms —
        staged one-shot, staged two-shot, registered in-place pull and push — at each size on
        this node, take every candidate's RANK-MAX time (``Comm.agree_max``, a host side
        channel), and set from it, identically on every rank:

        * ``oneshot_max``: the largest size up to which one-shot is at least as fast as
          two-shot (from the smallest size on);
        * ``auto_max``: the largest size up to which the better staged form beats RCCL (0 when
          RCCL wins already at the smallest size — ``auto`` then never uses the IPC kernel);
        * ``reg_max``: the same for the registered in-place forms (long-lived buffers).

        The table lands in :attr:`calibration` (result JSONs record it). Every candidate runs on
        fresh rank-seeded data and is checked against the fp32 sum once; a candidate that fails
        anywhere is dropped everywhere."""
        W, dev = self.comm.world_size, self.comm.device
        # every size a multiple of W 16-byte vectors, so two-shot is timed at each size for any W
        # (powers of two are not, at W = 3, 5, 6, 7)
        sizes = [int(n) - int(n) % (16 * W) for n in sizes if n <= self.capacity]
        sizes = [n for n in sizes if n > 0]
        table = []
        for n in sizes:
            g = torch.Generator(device=dev)
            g.manual_seed(4242 + self.comm.rank)
            x = torch.randn(n // 2, generator=g, device=dev).to(torch.bfloat16)
            ref = x.float()
            dist.all_reduce(ref)
            work = torch.empty_like(x)
            cands = {"rccl": lambda: dist.all_reduce(work)}
            if self.healthy and self.supports(x):
                cands["oneshot"] = lambda: self.all_reduce(x, work, algo=ONESHOT)
                if n % (8 * x.element_size() * W) == 0:
                    cands["twoshot"] = lambda: self.all_reduce(x, work, algo=TWOSHOT)
            rid = None
            if self.reg_healthy and self.supports_registered(work):
                rid = self.register(work)          # collective; released below
                cands["reg_pull"] = lambda: self.all_reduce_registered(work, rid)
                if self.push_healthy:
                    cands["reg_push"] = lambda: self.all_reduce_registered(work, rid, push=True)
            names = list(cands)
            ok = []
            for name in names:                 # correctness first, on every rank
                try:
                    work.copy_(x)
                    cands[name]()
                    torch.cuda.synchronize(dev)
                    good = bool(torch.allclose(work.float(), ref, rtol=2e-2, atol=5e-2 * W))
                    ok.append(1.0 if good and self.check_error() == 0 else 0.0)
                except Exception:  # noqa: BLE001 - a failed launch fails the candidate
                    ok.append(0.0)
            # passed everywhere = min over ranks = -(max over ranks of -passed)
            passed = [-v for v in self.comm.agree_max(names, [-v for v in ok])]
            times = [self._time_calls(cands[k], iters) if good > 0 else float("inf")
                     for k, good in zip(names, passed)]
            agreed = self.comm.agree_max(names, times)
            table.append({"bytes": n, "us": {k: (round(t * 1e6, 2) if t != float("inf")
                                                 else None) for k, t in zip(names, agreed)}})
            if rid is not None:
                self.deregister(rid)
        self._apply_calibration(table)
        return self.calibration

    def _apply_calibration(self, table) -> None:
        def t(row, k):
            v = row["us"].get(k)
            return float("inf") if v is None else v

        oneshot_max = 0
        twoshot_ran = any(row["us"].get("twoshot") is not None for row in table)
        for row in table:
            if row["us"].get("twoshot") is None and twoshot_ran:
                break       # not measured here: no evidence one-shot wins at this size
            if t(row, "oneshot") <= t(row, "twoshot"):
                oneshot_max = row["bytes"]
            else:
                break
        auto_max = 0
        for row in table:
            if min(t(row, "oneshot"), t(row, "twoshot")) < t(row, "rccl"):
                auto_max = row["bytes"]
            else:
                break
        reg_max = 0
        for row in table:
            if min(t(row, "reg_pull"), t(row, "reg_push")) < t(row, "rccl"):
                reg_max = row["bytes"]
            else:
                break
        if table:
            self.oneshot_max = oneshot_max
            self.auto_max = auto_max
        self.reg_max = reg_max
        self.calibration = {"world": self.comm.world_size, "table": table,
                            "oneshot_max": self.oneshot_max, "auto_max": self.auto_max,
                            "reg_max": reg_max, "agreed": "rank-max"}

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.dlbb_car_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def set_timeout_ms(ms: int) -> None:
    """Wall-clock bound of every IPC kernel's wait for its peers, for launches from now on
    (default 60000 ms; ``DLBB_CUSTOM_AR_TIMEOUT_MS``). A wait that exceeds it flags the error,
    later calls on that rank skip their waits (fail fast), and :meth:`CustomAllReduce.
    raise_if_error` raises on every rank."""
    _lib.lib().dlbb_car_set_timeout_ms(int(ms))


def get_custom_allreduce(comm: Comm, self_test: bool = True) -> Optional[CustomAllReduce]:
    """Process-wide instance (created collectively on first use). Returns None when disabled
    (``DLBB_CUSTOM_AR=0``) or unavailable."""
    if os.environ.get("DLBB_CUSTOM_AR", "1") == "0" or not comm.is_gpu:
        return None
    key = id(comm)
    if key not in _INSTANCES:
        cap = int(os.environ.get("DLBB_CUSTOM_AR_CAP", str(128 << 20)))
        if os.environ.get("DLBB_CUSTOM_AR_TIMEOUT_MS"):
            set_timeout_ms(int(os.environ["DLBB_CUSTOM_AR_TIMEOUT_MS"]))
        try:
            inst = CustomAllReduce(comm, capacity_bytes=cap)
            if self_test:
                inst.self_test()
                # the calibration's reference leg is the process group's all-reduce: only an
                # RCCL group gives the IPC-vs-RCCL crossover it is for. On a gloo group (ranks
                # sharing one GPU: tests, rehearsals) that leg is a host-staged CPU all-reduce of
                # up to 64 MiB x 20 iterations per rank — at 8 ranks 34.5 of a 38.8 s test
                # (round-5 probe, tools/diag/ipc8_probe.py), and the silent minutes that got an
                # 8-rank test killed in round 4 — and its crossovers would be meaningless
                if (comm.world_size > 1 and inst.healthy and comm.backend == "nccl"
                        and os.environ.get("DLBB_CUSTOM_AR_CALIBRATE", "1") != "0"):
                    inst.calibrate()
                elif comm.world_size > 1 and comm.backend != "nccl":
                    inst.calibration = {"world": comm.world_size, "skipped":
                                        f"process group is {comm.backend}, not RCCL: no "
                                        "crossover to measure (default thresholds)"}
        except RuntimeError as e:   # agreed on all ranks: fall back to RCCL everywhere
            if comm.rank == 0:
                print(f"[custom all-reduce disabled] {e}", flush=True)
            inst = None
        _INSTANCES[key] = inst
    return _INSTANCES[key]
