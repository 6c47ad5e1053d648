"""ctypes binding of the in-tree gfx950 kernel library ``_dlbb_hip.so``.

Loading order matters: torch is imported first so its bundled HIP runtime
(``torch/lib/libamdhip64.so``, SONAME ``libamdhip64.so.7``) is already mapped; our library's
``NEEDED libamdhip64.so.7`` then binds to that same runtime, so torch streams and device
pointers are valid inside our kernels (one HIP runtime per process).

Policy: on a GPU tensor the HIP kernel is the ONLY path — if the library is missing or a launch
fails, the op raises. A torch implementation is used only for CPU tensors (CPU plumbing /
unit tests) or when explicitly requested with ``DLBB_KERNELS=torch`` (A/B comparisons).
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

from .build import LIB_PATH, source_id

DT_F32, DT_BF16, DT_F16 = 0, 1, 2
_DT = {torch.float32: DT_F32, torch.bfloat16: DT_BF16, torch.float16: DT_F16}

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[BaseException] = None

c_void_p, c_int, c_int64, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float

_SIGS = {
    "dlbb_reduce_sum": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_int64, c_int, c_int,
                                c_float, c_void_p]),
    "dlbb_reduce_sum_grid": (c_int, [ctypes.POINTER(c_void_p), c_int, c_void_p, c_int64, c_int,
                                     c_int, c_float, c_int, c_void_p]),
    "dlbb_spin_ns": (c_int, [c_int64, c_int, c_void_p]),
    "dlbb_stamps_set": (None, [c_void_p, c_int64]),
    "dlbb_stamps_launches": (c_int64, []),
    "dlbb_stamps_entry": (c_int, [c_int64, ctypes.POINTER(c_int), ctypes.POINTER(c_int64),
                                  ctypes.POINTER(c_int64)]),
    "dlbb_cast": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int64, c_void_p]),
    "dlbb_pack_rows": (c_int, [c_void_p, c_int, c_int64, c_void_p, c_int, c_int64, c_int64,
                               c_int64, c_void_p]),
    "dlbb_chunk_copy": (c_int, [c_void_p, c_int64, c_void_p]),
    "dlbb_chunk_copy2": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "dlbb_chunk_copy_set_nt": (None, [c_int]),
    "dlbb_chunk_copy_scale": (c_int, [c_void_p, c_int64, c_int, c_int, c_float, c_void_p]),
    "dlbb_layernorm_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_int64, c_int, c_float,
                                   c_void_p]),
    "dlbb_layernorm_bwd_grid": (c_int, [c_int64]),
    "dlbb_layernorm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                   c_int, c_int, c_void_p]),
    "dlbb_bias_gelu_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                                   c_void_p]),
    "dlbb_bias_gelu_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                   c_int, c_int, c_void_p]),
    "dlbb_gemm_bf16_nt": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                  c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                  c_void_p, c_int, c_int, c_void_p]),
    "dlbb_gemm_bf16_nt_v": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                    c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                    c_void_p, c_int, c_int, c_int, c_void_p]),
    "dlbb_gemm_streamk_plan": (c_int, [c_int64, c_int64, c_int64, c_int, c_void_p]),
    "dlbb_gemm_bf16_nt_split": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                        c_int64, c_int64, c_int64, c_int, c_int, c_void_p,
                                        c_int64, c_void_p]),
    "dlbb_gemm_bf16_nt_streamk": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                          c_int64, c_int64, c_int64, c_int64, c_void_p,
                                          c_void_p, c_int64, c_void_p, c_int, c_int, c_int,
                                          c_void_p, c_int64, c_void_p, c_int64, c_void_p]),
    "dlbb_gemm_nt_phase_probe": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                         c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p]),
    "dlbb_gemm_bf16_nn": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                  c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                                  c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "dlbb_gemm_bf16_tn": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                  c_int64, c_int64, c_int64, c_void_p, c_int64, c_int, c_int,
                                  c_int, c_void_p, c_void_p]),
    "dlbb_gemm_set_tile": (None, [c_int]),
    "dlbb_gemm_set_stagger": (None, [c_int]),
    "dlbb_gemm_get_stagger": (c_int, []),
    "dlbb_gemm_set_bal": (None, [c_int]),
    "dlbb_gemm_set_persist_epi": (None, [c_int]),
    "dlbb_gemm_set_concurrent": (None, [c_int]),
    "dlbb_gemm_get_concurrent": (c_int, []),
    "dlbb_gemm_wgrad_set_stages": (None, [c_int]),
    "dlbb_attn_set_xcd": (None, [c_int]),
    "dlbb_attn_set_stamps": (None, [c_void_p, c_void_p, c_void_p]),
    "dlbb_xent_set_variant": (None, [c_int]),
    "dlbb_xent_count_inv": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "dlbb_xent_loss_mean": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "dlbb_xent_fused": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                                c_void_p, c_void_p]),
    "dlbb_adamw": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64,
                           c_float, c_float, c_float, c_float, c_float, c_int, c_float,
                           c_void_p]),
    "dlbb_adamw_devstep": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                   c_int64, c_float, c_float, c_float, c_float, c_float,
                                   c_void_p, c_float, c_void_p]),
    "dlbb_xent_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                              c_void_p]),
    "dlbb_xent_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                              c_void_p, c_void_p]),
    "dlbb_gemm_wgrad": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_int,
                                c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "dlbb_gemm_wgrad_tile": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int,
                                     c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                     c_int, c_void_p]),
    "dlbb_gemm_wgrad_tile2": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int,
                                     c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                     c_int, c_int, c_void_p]),
    "dlbb_gemm_wgrad_fused": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int,
                                      c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                      c_int, c_int, c_void_p, c_int, c_void_p]),
    "dlbb_gemm_wgrad_counters": (c_int, [c_int, c_int, c_int, c_int]),
    "dlbb_gemm_wgrad_set_order": (None, [c_int]),
    "dlbb_sort_ids": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "dlbb_stream_fork": (c_int, [c_void_p, c_void_p, c_int]),
    "dlbb_split_reduce": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_int64, c_int,
                                  c_int, c_void_p]),
    "dlbb_embedding_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                                   c_int64, c_void_p]),
    "dlbb_embedding_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                   c_int64, c_int, c_int, c_int64, c_void_p]),
    "dlbb_attn_fwd": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_int,
                              c_int, c_int, c_float, c_void_p]),
    "dlbb_attn_bwd": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p,
                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p]),
    "dlbb_rccl_unique_id_bytes": (c_int, []),
    "dlbb_rccl_get_unique_id": (c_int, [c_void_p]),
    "dlbb_rccl_init": (c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_void_p)]),
    "dlbb_rccl_run": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_int, c_int]),
    "dlbb_rccl_enqueue": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_int, c_int,
                                  c_void_p, c_int]),
    "dlbb_rccl_alltoallv": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int, c_void_p]),
    "dlbb_rccl_time_iters": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_int, c_int,
                                     c_int, c_int, ctypes.POINTER(ctypes.c_float)]),
    "dlbb_rccl_time_batched": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_int,
                                       c_int, c_int, c_int, ctypes.POINTER(ctypes.c_float)]),
    "dlbb_rccl_destroy": (c_int, [c_void_p]),
    "dlbb_car_create": (c_int, [c_int, c_int, c_int64, ctypes.POINTER(c_void_p)]),
    "dlbb_car_ipc_handles": (c_int, [c_void_p, c_void_p]),
    "dlbb_car_handle_bytes": (c_int, []),
    "dlbb_car_open": (c_int, [c_void_p, c_void_p, ctypes.POINTER(c_int)]),
    "dlbb_car_capacity": (c_int64, [c_void_p]),
    "dlbb_car_allreduce": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int,
                                   c_void_p]),
    "dlbb_car_reg_export": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_int64)]),
    "dlbb_car_reg_open": (c_int, [c_void_p, c_void_p, c_int64, c_void_p,
                                  ctypes.POINTER(c_int64), ctypes.POINTER(c_int)]),
    "dlbb_car_allreduce_reg": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p]),
    "dlbb_car_allreduce_reg_push": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p]),
    "dlbb_car_direct_reg": (c_int, [c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_int,
                                    c_void_p]),
    "dlbb_car_alltoallv_reg": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int64),
                                       ctypes.POINTER(c_int64), ctypes.POINTER(c_int64), c_void_p,
                                       c_int, c_void_p]),
    "dlbb_car_reg_close": (c_int, [c_void_p, c_int]),
    "dlbb_car_reg_counts": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "dlbb_car_open_local": (c_int, [ctypes.POINTER(c_void_p), c_int]),
    "dlbb_car_reg_local": (c_int, [ctypes.POINTER(c_void_p), c_int, ctypes.POINTER(c_void_p),
                                   c_int64, ctypes.POINTER(c_int)]),
    "dlbb_car_vr_max_blocks": (c_int, [c_int, c_int, c_int]),
    "dlbb_car_vr_launch": (c_int, [ctypes.POINTER(c_void_p), c_int, c_int,
                                   ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int64,
                                   c_int, c_int, c_int, c_void_p]),
    "dlbb_car_error": (c_int, [c_void_p]),
    "dlbb_car_set_timeout_ms": (None, [c_int]),
    "dlbb_car_destroy": (c_int, [c_void_p]),
}


class KernelError(RuntimeError):
    pass


def _load() -> ctypes.CDLL:
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        if _load_error is not None:
            raise KernelError(f"HIP kernel library unavailable: {_load_error}") from _load_error
        try:
            if not os.path.exists(LIB_PATH):
                raise FileNotFoundError(
                    f"{LIB_PATH} not built; run `python -m "
                    f"distributed_llm_backend_benchmark_amd.ops.build`")
            lib = ctypes.CDLL(LIB_PATH)
            check_build_id(lib, source_id())
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
            return lib
        except BaseException as e:  # remember and re-raise loudly on every use
            _load_error = e
            raise KernelError(f"HIP kernel library unavailable: {e}") from e


def check_build_id(lib, expected: str) -> str:
    """Raise unless the loaded library was built from exactly the csrc/ sources on disk (its
    ``dlbb_build_id()`` equals :func:`.build.source_id`): a stale binary must never be what a
    test or benchmark measures."""
    fn = getattr(lib, "dlbb_build_id", None)
    if fn is None:
        raise KernelError(f"{LIB_PATH} has no dlbb_build_id(): rebuild it")
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    got = fn().decode()
    if got != expected:
        raise KernelError(f"{LIB_PATH} was built from other sources (build id {got}, csrc/ on "
                          f"disk is {expected}): run `python -m "
                          "distributed_llm_backend_benchmark_amd.ops.build`")
    return got


def lib() -> ctypes.CDLL:
    return _load()


def available() -> bool:
    try:
        _load()
        return True
    except KernelError:
        return False


def loaded_path() -> Optional[str]:
    return LIB_PATH if _lib is not None else None


def force_torch() -> bool:
    return os.environ.get("DLBB_KERNELS", "hip").lower() == "torch"


def use_hip(*tensors: torch.Tensor) -> bool:
    """True when the HIP kernels must run: any tensor on the GPU (and not forced to torch)."""
    on_gpu = any(t is not None and t.is_cuda for t in tensors)
    if on_gpu and not force_torch():
        _load()  # raise loudly if the library is missing on a GPU box
        return True
    return False


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise KernelError(f"unsupported dtype {t.dtype}") from None


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


_HIP_ERRORS = {1: "hipErrorInvalidValue", 2: "hipErrorOutOfMemory", 3: "hipErrorNotInitialized",
               98: "hipErrorInvalidDeviceFunction", 209: "hipErrorNoBinaryForGpu",
               217: "hipErrorPeerAccessUnsupported", 400: "hipErrorInvalidHandle"}


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise KernelError(f"{what} failed: hip error {rc} ({_HIP_ERRORS.get(rc, '?')})")
