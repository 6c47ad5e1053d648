"""Communication layer: one torch.distributed process group (RCCL over xGMI / Gloo), the
collective op registry, the IPC xGMI all-reduce, tensor-parallel linears and the bucketed DDP
gradient all-reduce overlapped with backward."""

from .comm import Comm, init_distributed, resolve_backend
from .collectives import OPS, make_op, make_data, REFERENCE_1D_OPS, REFERENCE_3D_OPS

__all__ = ["Comm", "init_distributed", "resolve_backend", "OPS", "make_op", "make_data",
           "REFERENCE_1D_OPS", "REFERENCE_3D_OPS"]
