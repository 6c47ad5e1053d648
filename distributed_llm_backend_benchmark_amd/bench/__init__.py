"""Collective sweep engine (1D flat buffers, 3D activation shapes), timing loops and the
reference result schema."""

from . import schema
from .sweep import run_1d_sweep, run_3d_sweep
from .timing import time_per_iteration, time_batched

__all__ = ["schema", "run_1d_sweep", "run_3d_sweep", "time_per_iteration", "time_batched"]
