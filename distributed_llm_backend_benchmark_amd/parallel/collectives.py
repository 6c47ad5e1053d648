"""Collective op registry.

Every op the reference times plus ``reduce_scatter`` (absent from the reference,
required by BASELINE configs 3/5) and an MoE-shaped uneven ``alltoall_moe``:

================ ====================================== =========================================
op               reference call site                    here
================ ====================================== =========================================
allreduce        ``1d/openmpi.py:63``, ``1d/dsccl.py:65`` ``dist.all_reduce`` (RCCL) or the IPC xGMI
                                                          kernel (:mod:`.custom_allreduce`)
allgather        ``1d/openmpi.py:78``, ``1d/dsccl.py:76`` ``all_gather_into_tensor`` (one flat output,
                                                          no list staging); ``form="list"`` = ref
reduce_scatter   —                                      ``reduce_scatter_tensor``
broadcast        ``1d/openmpi.py:98``, ``1d/dsccl.py:87`` ``dist.broadcast`` root 0
reduce           ``1d/openmpi.py:148``, ``1d/dsccl.py:129`` ``dist.reduce`` root 0
gather           ``1d/openmpi.py:113``, ``1d/dsccl.py:102`` ``dist.gather`` root 0
scatter          ``1d/openmpi.py:134``, ``1d/dsccl.py:118`` ``dist.scatter`` root 0 (P copies of N)
alltoall         ``1d/openmpi.py:167``, ``1d/dsccl.py:143`` ``all_to_all_single``, equal N/P splits
alltoall_moe     —                                      uneven token splits (top-k router shaped);
                                                          ``direct`` = one-hop IPC pulls
sendrecv         ``1d/openmpi.py:189-193``                ring ``batch_isend_irecv``
================ ====================================== =========================================

``direct=True`` routes allgather / reduce_scatter / alltoall through the one-hop IPC kernels of
:mod:`.custom_allreduce` (every GPU pulls from all 7 peers at once over xGMI) instead of RCCL.

Each op separates ``reset()`` (restores in-place buffers, reference ``data.clone()`` at
``1d/dsccl.py:62``; never timed) from ``run()`` (the timed collective), reports its message
bytes, and can validate its result against a closed form computed from every rank's seeded
input (the reference never validates).
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops.elementwise import ChunkTable
from .comm import Comm

DTYPES = {
    "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
    "fp16": torch.float16, "float16": torch.float16,
    "fp32": torch.float32, "float32": torch.float32,
}
DTYPE_NAMES = {torch.bfloat16: "bfloat16", torch.float16: "float16", torch.float32: "float32"}


def make_data(shape, dtype: torch.dtype, rank: int, device: torch.device,
              seed: int = 42) -> torch.Tensor:
    """Rank-seeded normal data (reference ``torch.manual_seed(42 + rank)``,
    ``1d/dsccl.py:203-204``); generated on the device so no host staging is needed."""
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    return torch.randn(*shape, generator=g, device=device, dtype=torch.float32).to(dtype)


def _direct_ipc(comm: Comm, t: torch.Tensor, multiple: int):
    """(kernel object, registration id) for the direct IPC collectives on ``t`` (registered on
    every rank — collective). ``multiple``: element count granularity the kernel needs (16-byte
    vectors per chunk). Raises alike on every rank when unavailable."""
    if not (comm.is_gpu and comm.world_size > 1):
        raise RuntimeError("direct IPC collectives need world > 1 on HIP devices")
    if t.numel() % multiple:
        raise RuntimeError(f"direct IPC collective needs a multiple of {multiple} elements")
    from .custom_allreduce import get_custom_allreduce

    car = get_custom_allreduce(comm)
    if car is None or not car.reg_healthy:
        raise RuntimeError("IPC kernels unavailable or failed their self-test")
    return car, car.register(t)


class CollectiveOp:
    name = "base"
    in_place = False

    def __init__(self, comm: Comm, data: torch.Tensor, **opts):
        self.comm = comm
        self.data = data
        self.opts = opts
        self.P = comm.world_size
        self.rank = comm.rank
        self.setup()

    # ---- lifecycle
    def setup(self) -> None:
        pass

    def reset(self) -> None:
        pass

    def run(self) -> None:
        raise NotImplementedError

    def ipc_kernel(self):
        """The IPC collective instance this op launches (None: RCCL / gloo only)."""
        return getattr(self, "_custom", None) or getattr(self, "_car", None)

    def close(self) -> None:
        """Collective teardown: release IPC registrations this op made (every rank, same
        order). Safe to call twice; the op must not run afterwards."""
        car, rid = getattr(self, "_reg_owner", (None, None))
        if car is not None:
            self._reg_owner = (None, None)
            car.deregister(rid)

    # ---- accounting
    @property
    def message_bytes(self) -> int:
        return self.data.numel() * self.data.element_size()

    @property
    def num_elements(self) -> int:
        return self.data.numel()

    # ---- validation
    def expected(self, all_inputs: List[torch.Tensor]) -> Optional[torch.Tensor]:
        return None

    def result(self) -> Optional[torch.Tensor]:
        return None

    def check(self, all_inputs: List[torch.Tensor], rtol: float = 2e-2,
              atol: float = 5e-2) -> bool:
        exp = self.expected(all_inputs)
        got = self.result()
        if exp is None or got is None:
            return True
        return bool(torch.allclose(got.float(), exp.float(), rtol=rtol, atol=atol))


class AllReduce(CollectiveOp):
    name = "allreduce"
    in_place = True

    def setup(self):
        self.buf = self.data.clone()
        impl = self.opts.get("impl", "rccl")
        self._custom = None
        self._reg_id = None
        self._push = False
        self.nblocks = self.opts.get("nblocks")
        multi_gpu = self.comm.is_gpu and self.comm.world_size > 1
        if impl in ("custom", "custom_reg", "auto") and multi_gpu:
            from .custom_allreduce import get_custom_allreduce

            car = get_custom_allreduce(self.comm)
            if impl == "custom_reg":
                # in place on self.buf, IPC-mapped once on every rank (collective; raises on
                # every rank alike)
                if car is None or not car.reg_healthy or not car.supports_registered(self.buf):
                    raise RuntimeError("registered custom all-reduce unavailable for "
                                       f"{self.buf.numel()} x {self.buf.dtype}")
                self._push = bool(self.opts.get("push"))
                if self._push and (not car.push_healthy
                                   or self.buf.numel() * self.buf.element_size() > car.capacity):
                    raise RuntimeError("push-form registered all-reduce unavailable for "
                                       f"{self.buf.numel()} x {self.buf.dtype}")
                self._reg_id = car.register(self.buf)
                self._reg_owner = (car, self._reg_id)
                self._custom = car
            elif impl == "custom":
                if car is None or not car.healthy:
                    raise RuntimeError("custom all-reduce unavailable or failed its self-test")
                if not car.supports(self.buf):
                    raise RuntimeError(
                        f"custom all-reduce cannot take {self.buf.numel()} x {self.buf.dtype}")
                self._custom = car
            elif car is not None and car.should_use(self.buf):
                self._custom = car
        self.algo = self.opts.get("algo")
        self.impl = ("custom_reg" if self._reg_id is not None
                     else "custom" if self._custom is not None else "rccl")

    def reset(self):
        self.buf.copy_(self.data)

    def run(self):
        if self._reg_id is not None:
            self._custom.all_reduce_registered(self.buf, self._reg_id, nblocks=self.nblocks,
                                               push=self._push)
        elif self._custom is not None:
            self._custom.all_reduce_(self.buf, algo=self.algo, nblocks=self.nblocks)
        else:
            dist.all_reduce(self.buf, op=dist.ReduceOp.SUM)

    def expected(self, all_inputs):
        acc = torch.zeros_like(all_inputs[0], dtype=torch.float32)
        for x in all_inputs:
            acc += x.float()
        return acc

    def result(self):
        return self.buf


class AllGather(CollectiveOp):
    name = "allgather"

    def setup(self):
        self.form = self.opts.get("form", "tensor")
        n = self.data.numel()
        self._car = None
        if self.form == "list":
            # reference: dist.all_gather into a Python list (collectives/1d/dsccl.py:72-76). Here
            # ONE all_gather_into_tensor into a flat staging buffer, then the list unpack is one
            # chunk-copy launch over a (flat slice -> list entry) table (csrc/flatten.hip)
            self.outs = [torch.empty_like(self.data) for _ in range(self.P)]
            self.flat = self.data.reshape(-1)
            self.stage = torch.empty(self.P * n, dtype=self.data.dtype, device=self.data.device)
            self._unpack = ChunkTable([(self.stage[i * n:(i + 1) * n], o.reshape(-1))
                                       for i, o in enumerate(self.outs)])
            self._tensor_ok = True
            # the substitution is recorded in every result (op_impl), so the stats never label
            # it as the reference's list collective (parity unpinned: no fixture times both)
            self.impl = "allgather_into_tensor+unpack"
        else:
            self.out = torch.empty(self.P * n, dtype=self.data.dtype, device=self.data.device)
            self.flat = self.data.reshape(-1)
            self._tensor_ok = True
            if self.opts.get("direct"):     # direct one-hop pulls over xGMI
                self._car, self._rid = _direct_ipc(self.comm, self.flat,
                                                   16 // self.data.element_size())
                self._reg_owner = (self._car, self._rid)
                self.impl = "custom"

    def run(self):
        if self._car is not None:
            self._car.all_gather_registered(self.flat, self._rid, self.out,
                                            nblocks=self.opts.get("nblocks"))
            return
        if self.form == "list":
            if self._tensor_ok:
                try:
                    dist.all_gather_into_tensor(self.stage, self.flat)
                    self._unpack.run()
                    return
                except (RuntimeError, NotImplementedError, ValueError):
                    self._tensor_ok = False    # backend without _allgather_base
            dist.all_gather(self.outs, self.data)
            return
        if self._tensor_ok:
            try:
                dist.all_gather_into_tensor(self.out, self.flat)
                return
            except (RuntimeError, NotImplementedError, ValueError):
                # e.g. gloo without _allgather_base: list form into views of the flat output
                self._tensor_ok = False
        dist.all_gather(list(self.out.chunk(self.P)), self.flat)

    def expected(self, all_inputs):
        return torch.cat([x.reshape(-1).float() for x in all_inputs])

    def result(self):
        if self.form == "list":
            return torch.cat([o.reshape(-1) for o in self.outs])
        return self.out


class ReduceScatter(CollectiveOp):
    name = "reduce_scatter"

    def setup(self):
        n = self.data.numel() - self.data.numel() % self.P   # trim to a multiple of P
        self.inp = self.data.reshape(-1)[:n].contiguous()
        self.out = torch.empty(n // self.P, dtype=self.data.dtype, device=self.data.device)
        self._native = True
        self._car = None
        if self.opts.get("direct"):
            # the kernel reduces 8-element vectors of each rank's 1/P share
            self._car, self._rid = _direct_ipc(self.comm, self.inp, 8 * self.P)
            self._reg_owner = (self._car, self._rid)
            self.impl = "custom"

    @property
    def message_bytes(self):
        return self.inp.numel() * self.inp.element_size()

    def run(self):
        if self._car is not None:
            self._car.reduce_scatter_registered(self.inp, self._rid, self.out,
                                                nblocks=self.opts.get("nblocks"))
            return
        if self._native:
            try:
                dist.reduce_scatter_tensor(self.out, self.inp, op=dist.ReduceOp.SUM)
                return
            except (RuntimeError, NotImplementedError, ValueError):
                self._native = False  # gloo: emulate (documented, CPU plumbing only)
        tmp = self.inp.clone()
        dist.all_reduce(tmp)
        self.out.copy_(tmp.chunk(self.P)[self.rank])

    def expected(self, all_inputs):
        n = self.inp.numel()
        acc = sum(x.reshape(-1)[:n].float() for x in all_inputs)
        return acc.chunk(self.P)[self.rank]

    def result(self):
        return self.out


class Broadcast(CollectiveOp):
    name = "broadcast"
    in_place = True

    def setup(self):
        self.buf = self.data.clone()

    def reset(self):
        self.buf.copy_(self.data)

    def run(self):
        dist.broadcast(self.buf, src=0)

    def expected(self, all_inputs):
        return all_inputs[0].float()

    def result(self):
        return self.buf


class Reduce(CollectiveOp):
    name = "reduce"
    in_place = True

    def setup(self):
        self.buf = self.data.clone()

    def reset(self):
        self.buf.copy_(self.data)

    def run(self):
        dist.reduce(self.buf, dst=0, op=dist.ReduceOp.SUM)

    def expected(self, all_inputs):
        if self.rank != 0:
            return None
        return sum(x.float() for x in all_inputs)

    def result(self):
        return self.buf if self.rank == 0 else None


class Gather(CollectiveOp):
    name = "gather"

    def setup(self):
        self.glist = ([torch.empty_like(self.data) for _ in range(self.P)]
                      if self.rank == 0 else None)

    def run(self):
        dist.gather(self.data, gather_list=self.glist, dst=0)

    def expected(self, all_inputs):
        return torch.cat([x.reshape(-1).float() for x in all_inputs]) if self.rank == 0 else None

    def result(self):
        return torch.cat([g.reshape(-1) for g in self.glist]) if self.rank == 0 else None


class Scatter(CollectiveOp):
    name = "scatter"

    def setup(self):
        # reference: root holds P copies of its N-element buffer (1d/dsccl.py:110-113)
        self.slist = [self.data.clone() for _ in range(self.P)] if self.rank == 0 else None
        self.out = torch.empty_like(self.data)

    def run(self):
        dist.scatter(self.out, self.slist, src=0)

    def expected(self, all_inputs):
        return all_inputs[0].float()

    def result(self):
        return self.out


class AllToAll(CollectiveOp):
    name = "alltoall"

    def setup(self):
        n = self.data.numel() - self.data.numel() % self.P
        self.inp = self.data.reshape(-1)[:n].contiguous()
        self.out = torch.empty_like(self.inp)
        self._car = None
        if self.opts.get("direct"):
            self._car, self._rid = _direct_ipc(self.comm, self.inp,
                                               16 // self.inp.element_size() * self.P)
            self._reg_owner = (self._car, self._rid)
            self.impl = "custom"

    @property
    def message_bytes(self):
        return self.inp.numel() * self.inp.element_size()

    def run(self):
        if self._car is not None:
            self._car.all_to_all_registered(self.inp, self._rid, self.out,
                                            nblocks=self.opts.get("nblocks"))
            return
        dist.all_to_all_single(self.out, self.inp)

    def expected(self, all_inputs):
        n = self.inp.numel()
        c = n // self.P
        return torch.cat([x.reshape(-1)[:n][self.rank * c:(self.rank + 1) * c].float()
                          for x in all_inputs])

    def result(self):
        return self.out


def moe_split_sizes(tokens: int, world: int, hidden: int, seed: int = 7,
                    skew: float = 1.0) -> List[List[int]]:
    """Deterministic MoE-shaped send matrix ``S[src][dst]`` in ELEMENTS (tokens × hidden):
    each source routes ``tokens`` rows over ``world`` expert ranks with a Zipf-like skew, the
    shape a top-k router produces. Every rank computes the same matrix, so the uneven
    ``all_to_all_single`` splits are consistent without an extra exchange."""
    g = torch.Generator().manual_seed(seed)
    mat = []
    for src in range(world):
        w = torch.tensor([1.0 / ((d - src) % world + 1) ** skew for d in range(world)])
        w = w * (0.75 + 0.5 * torch.rand(world, generator=g))
        cnt = torch.floor(w / w.sum() * tokens).long()
        cnt[src] += tokens - int(cnt.sum())
        mat.append([int(c) * hidden for c in cnt])
    return mat


class AllToAllMoE(CollectiveOp):
    """Expert-parallel dispatch: ``data`` is ``[tokens, hidden]`` per rank; uneven splits from
    :func:`moe_split_sizes` (BASELINE config 4)."""

    name = "alltoall_moe"

    def setup(self):
        hidden = self.data.shape[-1]
        tokens = self.data.numel() // hidden
        self.mat = moe_split_sizes(tokens, self.P, hidden, seed=self.opts.get("moe_seed", 7))
        self.in_splits = self.mat[self.rank]
        self.out_splits = [self.mat[s][self.rank] for s in range(self.P)]
        self.inp = self.data.reshape(-1)
        self.out = torch.empty(sum(self.out_splits), dtype=self.data.dtype,
                               device=self.data.device)
        self._car = None
        if self.opts.get("direct"):
            # one-hop pulls over xGMI: this rank's tokens from every peer's registered input at
            # once (parallel/custom_allreduce.py all_to_allv_registered)
            if (hidden * self.data.element_size()) % 16:
                raise RuntimeError("direct MoE all-to-all needs 16-byte token rows")
            self._car, self._rid = _direct_ipc(self.comm, self.inp, 16 // self.data.element_size())
            self._reg_owner = (self._car, self._rid)
            me = self.rank
            self._src = [sum(self.mat[p][:me]) for p in range(self.P)]
            self._dst = [sum(self.out_splits[:p]) for p in range(self.P)]
            self.impl = "custom"

    def run(self):
        if self._car is not None:
            self._car.all_to_allv_registered(self.inp, self._rid, self.out, self._src,
                                             self.out_splits, self._dst,
                                             nblocks=self.opts.get("nblocks"))
            return
        dist.all_to_all_single(self.out, self.inp, output_split_sizes=self.out_splits,
                               input_split_sizes=self.in_splits)

    def expected(self, all_inputs):
        parts = []
        for s, x in enumerate(all_inputs):
            off = sum(self.mat[s][:self.rank])
            parts.append(x.reshape(-1)[off: off + self.mat[s][self.rank]].float())
        return torch.cat(parts)

    def result(self):
        return self.out


class SendRecv(CollectiveOp):
    name = "sendrecv"

    def setup(self):
        self.recv = torch.empty_like(self.data)
        self.nxt = (self.rank + 1) % self.P
        self.prv = (self.rank - 1 + self.P) % self.P

    def run(self):
        if self.P == 1:
            self.recv.copy_(self.data)
            return
        ops = [dist.P2POp(dist.isend, self.data, self.nxt),
               dist.P2POp(dist.irecv, self.recv, self.prv)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()

    def expected(self, all_inputs):
        return all_inputs[self.prv].float()

    def result(self):
        return self.recv


OPS: Dict[str, Callable[..., CollectiveOp]] = {
    c.name: c for c in (AllReduce, AllGather, ReduceScatter, Broadcast, Reduce, Gather,
                        Scatter, AllToAll, AllToAllMoE, SendRecv)
}

REFERENCE_1D_OPS = ["allreduce", "allgather", "broadcast", "gather", "scatter", "reduce",
                    "alltoall", "sendrecv"]
REFERENCE_3D_OPS = ["allreduce", "allgather", "broadcast", "gather", "reduce"]


def make_op(name: str, comm: Comm, data: torch.Tensor, **opts) -> CollectiveOp:
    if name not in OPS:
        raise KeyError(f"unknown collective {name!r}; known: {sorted(OPS)}")
    if opts.get("impl") == "native":
        # our own RCCL communicator driven from C++, enqueued on the caller's stream
        from .rccl_native import NATIVE_OPS

        if name not in NATIVE_OPS:
            raise KeyError(f"no native RCCL implementation of {name!r}")
        return NATIVE_OPS[name](comm, data, **opts)
    return OPS[name](comm, data, **opts)
