"""Native RCCL engine: our own RCCL communicator driven from C++ (``csrc/rccl_engine.hip``).

Why: torch's ProcessGroupNCCL enqueues every collective on an internal stream and joins it back
to the caller's stream with events — two extra dependencies per call that show up in small-
message latency, and a watchdog thread that makes RCCL calls un-capturable into HIP graphs on
this stack. The native engine owns a second communicator (``ncclCommInitRank`` with a unique id
that rank 0 creates and the torch process group broadcasts) and enqueues collectives directly
on the caller's stream, so

* the per-iteration device time is the RCCL kernel itself (reference methodology: barrier →
  timed call, ``collectives/1d/openmpi.py:60-65``),
* a loop of collectives can be captured into a HIP graph (``bench.timing.graph_safe``),
* ``time_iters`` / ``time_batched`` run the whole warmup + timed loop in C++ (nccl-tests).

Ops use the same semantics and validation as :mod:`.collectives` (subclasses that only replace
``setup``/``run``); select them with ``make_op(name, comm, data, impl="native")``.
"""

from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from ..ops import _lib
from . import collectives as C
from .comm import Comm

OP_CODES = {"allreduce": 0, "allgather": 1, "reduce_scatter": 2, "broadcast": 3, "reduce": 4,
            "alltoall": 5, "sendrecv": 6, "gather": 7, "scatter": 8}

_ENGINES: Dict[int, "NativeRCCL"] = {}


class NativeRCCL:
    """One RCCL communicator over the ranks of ``comm`` (one GPU per rank)."""

    def __init__(self, comm: Comm):
        if not comm.is_gpu:
            raise RuntimeError("native RCCL engine needs HIP devices")
        self.comm = comm
        self.lib = _lib.lib()
        self.h = None
        uid, err = None, None
        if comm.rank == 0:
            buf = ctypes.create_string_buffer(int(self.lib.dlbb_rccl_unique_id_bytes()))
            rc = self.lib.dlbb_rccl_get_unique_id(buf)
            uid, err = (bytes(buf.raw), None) if rc == 0 else (None, f"ncclGetUniqueId rc={rc}")
        uid, err = comm.broadcast_object((uid, err))
        if uid is None:
            raise RuntimeError(f"native RCCL setup failed: {err}")
        torch.cuda.set_device(comm.device)
        h = ctypes.c_void_p()
        rc = self.lib.dlbb_rccl_init(uid, comm.world_size, comm.rank, ctypes.byref(h))
        rcs = comm.all_gather_object(int(rc))
        if rc == 0:
            self.h = h
        if any(r != 0 for r in rcs):
            self.close()
            raise RuntimeError(f"ncclCommInitRank failed (rc per rank: {rcs}; 1000+ = "
                               "ncclResult_t)")

    # ------------------------------------------------------------------ enqueue / timing
    def enqueue(self, op: str, send: torch.Tensor, recv: torch.Tensor, count: int,
                root: int = 0, stream: Optional[int] = None) -> None:
        """Enqueue on ``stream`` (default: torch's current stream) without synchronising."""
        # NB: torch's default stream has handle 0 (the null stream) — a valid target, passed
        # through as is (the C side never reinterprets 0 as "engine stream")
        st = _lib.stream(send.device) if stream is None else stream
        rc = self.lib.dlbb_rccl_enqueue(self.h, OP_CODES[op], send.data_ptr(), recv.data_ptr(),
                                        int(count), _lib.dt(send), int(root), st, 0)
        if rc != 0:
            raise RuntimeError(f"native RCCL {op} failed: rc={rc}")

    def alltoallv(self, send: torch.Tensor, send_splits, recv: torch.Tensor, recv_splits,
                  stream: Optional[int] = None) -> None:
        """Uneven all-to-all: ``send_splits[p]`` elements go to peer p, ``recv_splits[p]``
        arrive from it (contiguous blocks in rank order), enqueued on ``stream``."""
        P = self.comm.world_size

        def arr(vals):
            return (ctypes.c_int64 * P)(*[int(v) for v in vals])

        def displs(splits):
            out, acc = [], 0
            for v in splits:
                out.append(acc)
                acc += int(v)
            return out

        st = _lib.stream(send.device) if stream is None else stream
        rc = self.lib.dlbb_rccl_alltoallv(self.h, send.data_ptr(), arr(send_splits),
                                          arr(displs(send_splits)), recv.data_ptr(),
                                          arr(recv_splits), arr(displs(recv_splits)),
                                          _lib.dt(send), st)
        if rc != 0:
            raise RuntimeError(f"native RCCL alltoallv failed: rc={rc}")

    def time_iters(self, op: str, send: torch.Tensor, recv: torch.Tensor, count: int,
                   iters: int, warmup: int, root: int = 0) -> List[float]:
        """Per-iteration device seconds, device barrier before each (C++ loop)."""
        torch.cuda.synchronize(send.device)
        out = (ctypes.c_float * max(1, iters))()
        rc = self.lib.dlbb_rccl_time_iters(self.h, OP_CODES[op], send.data_ptr(),
                                           recv.data_ptr(), int(count), _lib.dt(send),
                                           int(root), int(warmup), int(iters), out)
        if rc != 0:
            raise RuntimeError(f"native RCCL timing of {op} failed: rc={rc}")
        return [out[i] * 1e-6 for i in range(iters)]

    def time_batched(self, op: str, send: torch.Tensor, recv: torch.Tensor, count: int,
                     iters: int, warmup: int, root: int = 0) -> float:
        """Mean device seconds per call over ``iters`` back-to-back calls (C++ loop)."""
        torch.cuda.synchronize(send.device)
        out = ctypes.c_float()
        rc = self.lib.dlbb_rccl_time_batched(self.h, OP_CODES[op], send.data_ptr(),
                                             recv.data_ptr(), int(count), _lib.dt(send),
                                             int(root), int(warmup), int(iters),
                                             ctypes.byref(out))
        if rc != 0:
            raise RuntimeError(f"native RCCL batched timing of {op} failed: rc={rc}")
        return out.value * 1e-6

    def close(self) -> None:
        if self.h is not None:
            self.lib.dlbb_rccl_destroy(self.h)
            self.h = None


def get_native(comm: Comm) -> NativeRCCL:
    key = id(comm)
    eng = _ENGINES.get(key)
    if eng is None or eng.h is None:
        eng = NativeRCCL(comm)
        _ENGINES[key] = eng
    return eng


def close_all() -> None:
    for eng in _ENGINES.values():
        eng.close()
    _ENGINES.clear()


# ---------------------------------------------------------------------- ops
class _Native:
    impl = "native"
    code = ""

    def _engine(self) -> NativeRCCL:
        return get_native(self.comm)

    def native_args(self):
        """(send, recv, count, root) for the C++ engine."""
        raise NotImplementedError

    def run(self):
        send, recv, count, root = self.native_args()
        self.engine.enqueue(self.code, send, recv, count, root)


class NativeAllReduce(_Native, C.AllReduce):
    code = "allreduce"

    def setup(self):
        self.buf = self.data.clone()
        self.engine = self._engine()
        self.algo = None
        # out_of_place: result into a separate buffer (at one rank the collective is then a real
        # device copy instead of an empty call)
        self.out = torch.empty_like(self.buf) if self.opts.get("out_of_place") else self.buf

    def native_args(self):
        return self.buf, self.out, self.buf.numel(), 0

    def result(self):
        return self.out


class NativeAllGather(_Native, C.AllGather):
    code = "allgather"

    def setup(self):
        self.form = "tensor"
        self.flat = self.data.reshape(-1)
        self.out = torch.empty(self.P * self.flat.numel(), dtype=self.data.dtype,
                               device=self.data.device)
        self.engine = self._engine()

    def native_args(self):
        return self.flat, self.out, self.flat.numel(), 0


class NativeReduceScatter(_Native, C.ReduceScatter):
    code = "reduce_scatter"

    def setup(self):
        C.ReduceScatter.setup(self)
        self.engine = self._engine()

    def native_args(self):
        return self.inp, self.out, self.inp.numel(), 0


class NativeBroadcast(_Native, C.Broadcast):
    code = "broadcast"

    def setup(self):
        self.buf = self.data.clone()
        self.engine = self._engine()
        # out_of_place: root's data -> buf (at one rank a real device copy, not an empty call)
        self.src = self.data.reshape(-1) if self.opts.get("out_of_place") else self.buf

    def native_args(self):
        return self.src, self.buf, self.buf.numel(), 0


class NativeReduce(_Native, C.Reduce):
    code = "reduce"

    def setup(self):
        self.buf = self.data.clone()
        self.engine = self._engine()
        self.src = self.data.reshape(-1) if self.opts.get("out_of_place") else self.buf

    def native_args(self):
        return self.src, self.buf, self.buf.numel(), 0


class NativeGather(_Native, C.Gather):
    code = "gather"

    def setup(self):
        self.flat = self.data.reshape(-1)
        n = self.flat.numel()
        # recvbuff is only written on the root; others pass a 1-element placeholder
        self.out = torch.empty(self.P * n if self.rank == 0 else 1, dtype=self.data.dtype,
                               device=self.data.device)
        self.engine = self._engine()

    def native_args(self):
        return self.flat, self.out, self.flat.numel(), 0

    def result(self):
        return self.out if self.rank == 0 else None


class NativeScatter(_Native, C.Scatter):
    code = "scatter"

    def setup(self):
        # reference: root holds P copies of its N-element buffer (1d/dsccl.py:110-113)
        flat = self.data.reshape(-1)
        self.src = (flat.repeat(self.P) if self.rank == 0 else flat.clone())
        self.out = torch.empty_like(flat)
        self.engine = self._engine()

    def native_args(self):
        return self.src, self.out, self.out.numel(), 0

    def result(self):
        return self.out.view_as(self.data)


class NativeAllToAll(_Native, C.AllToAll):
    code = "alltoall"

    def setup(self):
        C.AllToAll.setup(self)
        self.engine = self._engine()

    def native_args(self):
        return self.inp, self.out, self.inp.numel(), 0


class NativeSendRecv(_Native, C.SendRecv):
    code = "sendrecv"

    def setup(self):
        C.SendRecv.setup(self)
        self.flat = self.data.reshape(-1)
        self.engine = self._engine()

    def native_args(self):
        return self.flat, self.recv.view(-1), self.flat.numel(), 0


class NativeAllToAllMoE(_Native, C.AllToAllMoE):
    """Uneven MoE-shaped all-to-all (``ncclAllToAllv``) with the registry op's split matrix."""

    code = "alltoall_moe"

    def setup(self):
        C.AllToAllMoE.setup(self)
        self.engine = self._engine()

    def run(self):
        self.engine.alltoallv(self.inp, self.in_splits, self.out, self.out_splits)


NATIVE_OPS = {c.code: c for c in (NativeAllToAllMoE, NativeAllReduce, NativeAllGather, NativeReduceScatter,
                                  NativeBroadcast, NativeReduce, NativeGather, NativeScatter,
                                  NativeAllToAll, NativeSendRecv)}
