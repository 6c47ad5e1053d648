"""Memory-bound ops: n-way reduce, cast, strided pack, multi-tensor chunk copy.

GPU tensors run the gfx950 kernels in ``csrc/reduce.hip``, ``csrc/cast.hip``,
``csrc/flatten.hip``; CPU tensors use the equivalent torch expression (plumbing/tests).
"""

from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import check, dt, ptr, stream, use_hip

MAX_REDUCE_SRCS = 16


def spin_ns(ns: int, nblocks: int, device=None) -> None:
    """Hold ``nblocks`` workgroup slots for ``ns`` nanoseconds on the current stream (the
    link-bound duration of an emulated collective, ``csrc/reduce.hip`` spin_kernel)."""
    dev = device or torch.device("cuda", torch.cuda.current_device())
    check(_lib.lib().dlbb_spin_ns(int(ns), int(nblocks), stream(dev)), "spin_ns")


def reduce_sum(srcs: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None,
               out_dtype: Optional[torch.dtype] = None, scale: float = 1.0,
               nblocks: Optional[int] = None) -> torch.Tensor:
    """``out = scale * sum(srcs)`` with fp32 accumulation (the local SUM of an all-reduce).
    ``nblocks`` caps the kernel's grid (a CU budget when it runs beside compute)."""
    if not srcs:
        raise ValueError("reduce_sum needs at least one source")
    n = srcs[0].numel()
    for s in srcs:
        if s.numel() != n or s.dtype != srcs[0].dtype or not s.is_contiguous():
            raise ValueError("reduce_sum sources must be contiguous, same numel and dtype")
    if out is None:
        out = torch.empty(srcs[0].shape, dtype=out_dtype or srcs[0].dtype,
                          device=srcs[0].device)
    if use_hip(*srcs, out):
        if len(srcs) > MAX_REDUCE_SRCS:
            part = reduce_sum(srcs[:MAX_REDUCE_SRCS], out_dtype=torch.float32)
            return reduce_sum([part.to(srcs[0].dtype)] + list(srcs[MAX_REDUCE_SRCS:]), out,
                              scale=scale)
        arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
        check(_lib.lib().dlbb_reduce_sum_grid(arr, len(srcs), out.data_ptr(), n, dt(srcs[0]),
                                              dt(out), float(scale), int(nblocks or 0),
                                              stream(out.device)), "reduce_sum")
        return out
    acc = torch.zeros(srcs[0].shape, dtype=torch.float32, device=srcs[0].device)
    for s in srcs:
        acc += s.float()
    out.copy_(acc * scale if scale != 1.0 else acc)
    return out


def cast(x: torch.Tensor, dtype: torch.dtype, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Contiguous dtype conversion (bf16/fp16/fp32)."""
    if out is None:
        out = torch.empty(x.shape, dtype=dtype, device=x.device)
    if use_hip(x, out):
        xc = x if x.is_contiguous() else x.contiguous()
        check(_lib.lib().dlbb_cast(xc.data_ptr(), dt(xc), out.data_ptr(), dt(out), xc.numel(),
                                   stream(out.device)), "cast")
        return out
    out.copy_(x.to(dtype))
    return out


def pack_rows(x: torch.Tensor, out: Optional[torch.Tensor] = None,
              dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Dense copy (+cast) of a 2-D view with unit column stride and any row stride, e.g.
    ``qkv[..., :h]`` -> contiguous ``[rows, h]`` in one pass."""
    x2 = x.reshape(-1, x.shape[-1]) if x.dim() != 2 else x
    if x2.stride(-1) != 1:
        raise ValueError("pack_rows needs unit stride along the last dim")
    rows, cols = x2.shape
    if out is None:
        out = torch.empty(x.shape, dtype=dtype or x.dtype, device=x.device)
    if use_hip(x, out):
        check(_lib.lib().dlbb_pack_rows(x2.data_ptr(), dt(x2), x2.stride(0), out.data_ptr(),
                                        dt(out), cols, rows, cols, stream(out.device)),
              "pack_rows")
        return out
    out.copy_(x.to(out.dtype))
    return out


class ChunkTable:
    """A device-resident (src, dst, nbytes) copy list executed by ONE kernel launch.

    Built once per layout (e.g. a gradient bucket) and replayed every step; chunks are capped
    at ``chunk_bytes`` so one workgroup moves one chunk and large tensors spread over the GPU.
    """

    def __init__(self, pairs: Sequence[Tuple[torch.Tensor, torch.Tensor]],
                 chunk_bytes: int = 256 * 1024):
        rows: List[Tuple[int, int, int]] = []
        self.pairs = list(pairs)
        dev = None
        for src, dst in self.pairs:
            if src.numel() * src.element_size() != dst.numel() * dst.element_size():
                raise ValueError("chunk copy: src/dst byte sizes differ")
            if not (src.is_contiguous() and dst.is_contiguous()):
                raise ValueError("chunk copy: tensors must be contiguous")
            dev = src.device
            nb = src.numel() * src.element_size()
            s, d = src.data_ptr(), dst.data_ptr()
            off = 0
            while off < nb:
                c = min(chunk_bytes, nb - off)
                rows.append((s + off, d + off, c))
                off += c
        self.nchunks = len(rows)
        self.nbytes = sum(r[2] for r in rows)
        arr = np.asarray(rows if rows else [(0, 0, 0)], dtype=np.uint64)
        host = torch.from_numpy(arr.view(np.int64).copy())
        self.device = dev or torch.device("cpu")
        self.table = host.to(self.device) if self.device.type == "cuda" else host
        self.elem_pairs = [(s.numel(), s.dtype, d.dtype) for s, d in self.pairs]

    def run(self) -> None:
        if self.nchunks == 0:
            return
        if use_hip(self.table):
            check(_lib.lib().dlbb_chunk_copy2(self.table.data_ptr(), self.nchunks, self.nbytes,
                                              stream(self.device)), "chunk_copy")
            return
        for s, d in self.pairs:
            d.view(-1).view(torch.uint8).copy_(s.reshape(-1).view(torch.uint8))


def flatten_into(tensors: Sequence[torch.Tensor], flat: torch.Tensor) -> ChunkTable:
    """Build a table copying ``tensors`` back-to-back into ``flat`` (returns it; call
    ``.run()`` each time)."""
    pairs, off = [], 0
    f = flat.view(-1)
    for t in tensors:
        if t.dtype != flat.dtype or not t.is_contiguous():
            raise ValueError("flatten_into: tensors must be contiguous and match the flat dtype")
        n = t.numel()
        pairs.append((t.view(-1), f[off:off + n]))
        off += n
    if off > f.numel():
        raise ValueError("flatten_into: flat buffer too small")
    return ChunkTable(pairs)


def unflatten_scale(flat_views: Sequence[torch.Tensor], tensors: Sequence[torch.Tensor],
                    scale: float) -> None:
    """``tensors[i] = scale * flat_views[i]`` (dtype may change) — torch fallback only used on
    CPU; the GPU path is :class:`ScaleTable`."""
    for s, d in zip(flat_views, tensors):
        d.copy_((s.float() * scale).to(d.dtype).view_as(d))


class ScaleTable(ChunkTable):
    """Chunk table whose copies multiply by ``scale`` (e.g. 1/world gradient averaging) and may
    convert dtype; element sizes are taken from the src/dst dtypes."""

    def __init__(self, pairs, scale: float, chunk_elems: int = 65536):
        self.scale = float(scale)
        rows = []
        self.pairs = list(pairs)
        dev = None
        self.dt_in = self.dt_out = None
        for src, dst in self.pairs:
            if src.numel() != dst.numel():
                raise ValueError("scale copy: numel differs")
            dev = src.device
            self.dt_in, self.dt_out = src.dtype, dst.dtype
            es, ed = src.element_size(), dst.element_size()
            n = src.numel()
            off = 0
            while off < n:
                c = min(chunk_elems, n - off)
                rows.append((src.data_ptr() + off * es, dst.data_ptr() + off * ed, c * es))
                off += c
        self.nchunks = len(rows)
        self.nbytes = sum(r[2] for r in rows)
        arr = np.asarray(rows if rows else [(0, 0, 0)], dtype=np.uint64)
        host = torch.from_numpy(arr.view(np.int64).copy())
        self.device = dev or torch.device("cpu")
        self.table = host.to(self.device) if self.device.type == "cuda" else host

    def run(self) -> None:
        if self.nchunks == 0:
            return
        if use_hip(self.table):
            check(_lib.lib().dlbb_chunk_copy_scale(
                self.table.data_ptr(), self.nchunks, _lib._DT[self.dt_in], _lib._DT[self.dt_out],
                self.scale, stream(self.device)), "chunk_copy_scale")
            return
        for s, d in self.pairs:
            d.copy_((s.float() * self.scale).to(d.dtype).view_as(d))
