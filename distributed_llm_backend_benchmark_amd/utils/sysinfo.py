"""System / device / library information (reference ``utils.py:132-151``, extended with GPU,
ROCm and RCCL versions as SURVEY §5.5 asks)."""

from __future__ import annotations

import os
import platform
from typing import Dict, Any


def collect_system_info(include_gpu: bool = True) -> Dict[str, Any]:
    import psutil
    import torch

    info: Dict[str, Any] = {
        "platform": platform.platform(),
        "python_version": platform.python_version(),
        "torch_version": torch.__version__,
        "cpu_count": psutil.cpu_count(logical=False),
        "cpu_count_logical": psutil.cpu_count(logical=True),
        "total_memory_gb": psutil.virtual_memory().total / (1024 ** 3),
        "hip_version": getattr(torch.version, "hip", None),
    }
    if include_gpu:
        try:
            if torch.cuda.is_available():
                idx = torch.cuda.current_device()
                p = torch.cuda.get_device_properties(idx)
                info.update({
                    "gpu_name": p.name,
                    "gpu_arch": getattr(p, "gcnArchName", None),
                    "gpu_count": torch.cuda.device_count(),
                    "gpu_memory_gb": p.total_memory / (1024 ** 3),
                    "gpu_cu_count": p.multi_processor_count,
                })
                try:
                    v = torch.cuda.nccl.version()
                    info["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
                except Exception:
                    pass
        except Exception as e:  # never fail a run on info collection
            info["gpu_info_error"] = repr(e)
    for k in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS",
              "RCCL_MSCCL_ENABLE", "HIP_VISIBLE_DEVICES", "OMP_NUM_THREADS"):
        if k in os.environ:
            info.setdefault("env", {})[k] = os.environ[k]
    return info
