"""Config schema (reference config/baseline_config.yaml) and result-file naming."""

import os

import pytest
import yaml

from conftest import REPO
from distributed_llm_backend_benchmark_amd.bench import schema
from distributed_llm_backend_benchmark_amd.utils.config import (ConfigError, load_config,
                                                                validate_config)

REF_CFG = {
    "experiment": {"name": "baseline_7b_world4", "output_dir": "results"},
    "model": {"size": "7B", "hidden_size": 4096, "num_layers": 32, "num_heads": 32,
              "ffn_intermediate": 16384},
    "parallelism": {"world_size": 4, "cores_per_rank": 14},
    "input": {"batch_size": 8, "sequence_length": 512, "seed": 42},
    "execution": {"warmup_iterations": 5, "benchmark_iterations": 10},
    "system": {"omp_num_threads": 14, "mkl_num_threads": 14},
}


def test_reference_config_verbatim_is_accepted(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(REF_CFG))
    cfg = load_config(str(p))
    assert cfg["model"]["hidden_size"] == 4096
    assert cfg["execution"]["allreduce"] == "auto"        # additions get defaults
    assert cfg["execution"]["attention"] == "slice"


@pytest.mark.parametrize("name", ["baseline_config.yaml", "1b_config.yaml", "7b_config.yaml",
                                  "13b_config.yaml"])
def test_shipped_configs_load(name):
    cfg = load_config(os.path.join(REPO, "config", name))
    assert set(cfg) >= {"experiment", "model", "parallelism", "input", "execution", "system"}


def test_config_errors():
    bad = {k: dict(v) for k, v in REF_CFG.items()}
    del bad["model"]["hidden_size"]
    with pytest.raises(ConfigError):
        validate_config(bad)
    bad = {k: dict(v) for k, v in REF_CFG.items()}
    bad["execution"]["allreduce"] = "mpi"
    with pytest.raises(ConfigError):
        validate_config(bad)


def test_reference_sizes_and_labels():
    s = schema.resolve_1d_sizes("reference", 2)
    assert list(s.items()) == [("1KB", 256), ("64KB", 16384), ("1MB", 262144),
                               ("16MB", 4194304)]
    sw = schema.resolve_1d_sizes("sweep", 2)
    assert list(sw)[0] == "1KiB" and list(sw)[-1] == "1GiB" and sw["1GiB"] == (1 << 29)
    assert schema.resolve_1d_sizes("4KiB:16KiB", 4) == {"4KiB": 1024, "8KiB": 2048,
                                                          "16KiB": 4096}
    assert schema.resolve_1d_sizes("1KB,512", 2) == {"1KB": 256, "512B": 256}
    assert schema.filename_1d("rccl", "allreduce", 8, "16MB") == "rccl_allreduce_ranks8_16MB.json"
    assert (schema.filename_3d("rccl", "allgather", 4, 8, 2048, 4096)
            == "rccl_allgather_ranks4_b8_s2048_h4096.json")


def test_result_3d_keys():
    r = schema.result_3d(impl="rccl", backend="rccl", op="allreduce", ranks=8, batch=8,
                         seq_len=2048, hidden_dim=2048, dtype="bfloat16", wire_dtype="bfloat16",
                         wire_bytes=64 << 20, warmup=10, iters=100, timing_method="hip_event",
                         timings=[[0.1]])
    ref_keys = {"implementation", "backend", "operation", "num_ranks", "tensor_shape",
                "num_elements", "tensor_size_bytes", "tensor_size_mb", "dtype",
                "warmup_iterations", "measurement_iterations", "timing_method", "timings"}
    assert ref_keys <= set(r)
    assert r["tensor_size_mb"] == 64.0
