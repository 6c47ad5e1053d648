"""MI355X-native distributed collective / LLM-communication benchmark framework.

Capabilities mirror ``hardik-jinda/distributed-llm-backend-benchmark``:

* 1D flat-buffer and 3D activation-shaped collective sweeps (``bench``),
  with ``[rank][iter]`` timing matrices written in the reference's JSON schema
  (reference ``collectives/1d/openmpi.py:275-285``, ``collectives/3d/dsccl.py:207-225``).
* Offline statistics (``stats``) reproducing the reference CSV/JSON layouts
  (``collectives/1d/stats.py``, ``collectives/3d/stats.py``) plus nccl-tests busBW.
* A Megatron-style tensor-parallel transformer forward benchmark (``models.tp_transformer``,
  ``cli.run_tp``) with the reference's YAML schema (``config/baseline_config.yaml``).
* A GPT-2-small DDP training microbenchmark whose gradient-bucket all-reduce overlaps
  backward (``parallel.ddp``, ``models.gpt2``, ``cli.train_ddp``).

The four CPU backends of the reference (OpenMPI, Intel MPI, DeepSpeed+Gloo, DeepSpeed+oneCCL)
are replaced by one ``torch.distributed`` process group: RCCL (backend ``"nccl"`` on ROCm) over
xGMI on MI355X, Gloo for CPU plumbing. Hot ops are hand-written gfx950 HIP kernels under
``csrc/`` (n-way reduce, cast/pack, multi-tensor flatten, IPC xGMI all-reduce, MFMA GEMM,
fused residual+LayerNorm, bias-GELU, fused AdamW), loaded through ``ops``.
"""

__version__ = "0.1.0"

PACKAGE_NAME = "distributed_llm_backend_benchmark_amd"
