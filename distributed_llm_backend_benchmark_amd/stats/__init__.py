"""Offline statistics over sweep results (reference ``collectives/{1d,3d}/stats.py``)."""

from .bandwidth import (algbw_gbps, busbw_gbps, bus_factor, legacy_bandwidth_gbps, KNOWN_OPS)
from . import stats1d, stats3d

__all__ = ["algbw_gbps", "busbw_gbps", "bus_factor", "legacy_bandwidth_gbps", "KNOWN_OPS",
           "stats1d", "stats3d"]
