"""Native RCCL engine plumbing that can be checked without a GPU."""

import pytest
import torch


def test_native_ops_registry_and_cpu_refusal():
    from distributed_llm_backend_benchmark_amd.parallel import collectives as C
    from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
    from distributed_llm_backend_benchmark_amd.parallel.rccl_native import NATIVE_OPS, OP_CODES

    # every native op mirrors a registry op (same validation closed forms)
    for name, cls in NATIVE_OPS.items():
        assert name in C.OPS and issubclass(cls, C.OPS[name])
        assert name in OP_CODES or name == "alltoall_moe"      # alltoallv has its own entry
    comm = init_distributed("gloo")
    try:
        with pytest.raises(RuntimeError, match="HIP devices"):
            C.make_op("allreduce", comm, torch.ones(16), impl="native")
        with pytest.raises(KeyError):
            C.make_op("no_such_op", comm, torch.ones(4, 4), impl="native")
    finally:
        comm.destroy()


def test_native_symbols_exported():
    from distributed_llm_backend_benchmark_amd.ops import _lib

    lib = _lib.lib()
    assert lib.dlbb_rccl_unique_id_bytes() == 128
    for sym in ("dlbb_rccl_get_unique_id", "dlbb_rccl_init", "dlbb_rccl_enqueue",
                "dlbb_rccl_alltoallv",
                "dlbb_rccl_time_iters", "dlbb_rccl_time_batched", "dlbb_rccl_destroy"):
        assert hasattr(lib, sym)


def test_tracing_ranges_and_torch_profile(tmp_path):
    from distributed_llm_backend_benchmark_amd.utils import tracing

    with tracing.range("disabled"):          # no-op when disabled
        pass
    tracing.enable()
    try:
        with tracing.range("enabled"):
            tracing.mark("m")
    finally:
        tracing.enable(False)
    with tracing.torch_profile(str(tmp_path), rank=3):
        torch.ones(8).sum()
    assert (tmp_path / "trace_rank3.json").exists()
