"""IPC one-shot / two-shot xGMI all-reduce (``csrc/custom_allreduce.hip``).

The oneCCL algorithm sweep of the reference (``CCL_ALLREDUCE`` ∈ direct/ring/2d/...,
``collectives/3d/launch_dsccl.sh:46-47``) maps here to three all-reduce implementations on one
node: RCCL (ring/tree, default), ``oneshot`` (every rank reads all peers' full buffers over its
7 dedicated xGMI links — the "direct" analogue, lowest latency) and ``twoshot`` (direct
reduce-scatter + direct all-gather — the "2d"/rabenseifner analogue, all links busy).

Setup: each rank allocates its IPC regions, the 192-byte handles and device ordinals are
exchanged once through the process group (``all_gather_object``), peers are opened with
``hipIpcOpenMemHandle``. ``auto`` selection uses the custom kernel only below a crossover
size and only after a start-up self-test against RCCL passed on every rank.
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

from ..ops import _lib
from .comm import Comm

ONESHOT, TWOSHOT = 1, 2

_INSTANCES: Dict[int, "CustomAllReduce"] = {}


class CustomAllReduce:
    def __init__(self, comm: Comm, capacity_bytes: int = 64 << 20,
                 oneshot_max_bytes: int = 256 << 10, auto_max_bytes: int = 8 << 20,
                 nblocks: Optional[int] = None):
        if not comm.is_gpu:
            raise RuntimeError("custom all-reduce needs HIP devices")
        if comm.world_size > 8:
            raise RuntimeError("custom all-reduce supports up to 8 ranks (one node)")
        self.comm = comm
        self.lib = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(self.lib.dlbb_car_create(comm.rank, comm.world_size, int(capacity_bytes),
                                            ctypes.byref(h)), "car_create")
        self.h = h
        nb = self.lib.dlbb_car_handle_bytes()
        buf = ctypes.create_string_buffer(nb)
        _lib.check(self.lib.dlbb_car_ipc_handles(self.h, buf), "car_ipc_handles")
        mine = (bytes(buf.raw), torch.cuda.current_device())
        allh = comm.all_gather_object(mine)
        blob = b"".join(x[0] for x in allh)
        devs = (ctypes.c_int * comm.world_size)(*[int(x[1]) for x in allh])
        _lib.check(self.lib.dlbb_car_open(self.h, blob, devs), "car_open")
        self.capacity = int(self.lib.dlbb_car_capacity(self.h))
        self.oneshot_max = oneshot_max_bytes
        self.auto_max = auto_max_bytes
        self.nblocks = nblocks
        self.healthy = False

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
        # ~64 KiB of message per workgroup, 1..128 workgroups
        per = max(1, nbytes // (64 << 10))
        return int(min(128, max(1, per if algo == TWOSHOT else min(per, 32))))

    # ------------------------------------------------------------------ ops
    def all_reduce(self, inp: torch.Tensor, out: Optional[torch.Tensor] = None,
                   algo: Optional[int] = None) -> torch.Tensor:
        if not self.supports(inp):
            raise ValueError(f"custom all-reduce cannot take {inp.numel()} x {inp.dtype}")
        out = inp if out is None else out
        nbytes = inp.numel() * inp.element_size()
        a = algo or self.algo_for(nbytes, 8 * inp.element_size())
        _lib.check(self.lib.dlbb_car_allreduce(
            self.h, inp.data_ptr(), out.data_ptr(), inp.numel(), _lib.dt(inp), a,
            self.blocks_for(nbytes, a), _lib.stream(inp.device)), "car_allreduce")
        return out

    def all_reduce_(self, t: torch.Tensor, algo: Optional[int] = None) -> torch.Tensor:
        return self.all_reduce(t, t, algo)

    def check_error(self) -> int:
        return int(self.lib.dlbb_car_error(self.h))

    def self_test(self) -> bool:
        """Compare one-shot and two-shot against RCCL on small/medium messages; all ranks must
        pass for ``healthy``."""
        ok = True
        dev = self.comm.device
        for n in (4096, 1 << 18):
            g = torch.Generator(device=dev)
            g.manual_seed(1234 + self.comm.rank)
            x = torch.randn(n, generator=g, device=dev).to(torch.bfloat16)
            ref = x.float().clone()
            if self.comm.world_size > 1:
                dist.all_reduce(ref)
            for algo in (ONESHOT, TWOSHOT):
                y = self.all_reduce(x.clone(), algo=algo)
                torch.cuda.synchronize(dev)
                good = torch.allclose(y.float(), ref, rtol=2e-2, atol=5e-2 * self.comm.world_size)
                ok = ok and good and self.check_error() == 0
        flags = self.comm.all_gather_object(bool(ok))
        self.healthy = all(flags)
        return self.healthy

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.dlbb_car_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def get_custom_allreduce(comm: Comm, self_test: bool = True) -> Optional[CustomAllReduce]:
    """Process-wide instance (created collectively on first use). Returns None when disabled
    (``DLBB_CUSTOM_AR=0``) or unavailable."""
    if os.environ.get("DLBB_CUSTOM_AR", "1") == "0" or not comm.is_gpu:
        return None
    key = id(comm)
    inst = _INSTANCES.get(key)
    if inst is None:
        cap = int(os.environ.get("DLBB_CUSTOM_AR_CAP", str(64 << 20)))
        inst = CustomAllReduce(comm, capacity_bytes=cap)
        if self_test:
            inst.self_test()
        _INSTANCES[key] = inst
    return inst
