"""Shared experiment utilities: config, metrics/timing, JSON IO, system info.

Parity map (reference ``utils.py``): ``MetricsCollector`` (17-70), ``Timer`` (73-87),
``load_config`` (90-102), ``save_json``/``load_json`` (105-129), ``collect_system_info``
(132-151), ``setup_environment`` (154-169), ``print_summary`` (247-265),
``save_results`` (268-279).
"""

from .config import load_config, setup_environment, validate_config, DEFAULT_CONFIG
from .io import save_json, load_json, save_results
from .metrics import MetricsCollector, Timer, summarize
from .sysinfo import collect_system_info

__all__ = [
    "load_config", "setup_environment", "validate_config", "DEFAULT_CONFIG",
    "save_json", "load_json", "save_results",
    "MetricsCollector", "Timer", "summarize",
    "collect_system_info",
]
