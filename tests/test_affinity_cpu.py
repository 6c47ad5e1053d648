"""Per-rank NUMA binding plan (reference launch_openmpi.sh:19-23
``--bind-to core --map-by socket:PE=14`` and collectives/3d/launch_dsccl.sh:69-74 with
config_8.txt) on a fake sysfs tree: 8 GPUs on 2 NUMA nodes, 8 local ranks."""

import os

import pytest

from distributed_llm_backend_benchmark_amd.utils import affinity as A

NODE_CPUS = {0: "0-55,112-167", 1: "56-111,168-223"}


def _fake_sysfs(root):
    bdfs = {}
    for d in range(8):
        bdf = f"0000:{0x11 + 0x20 * d:02x}:00.0"
        bdfs[d] = bdf
        base = root / "bus" / "pci" / "devices" / bdf
        base.mkdir(parents=True)
        node = 0 if d < 4 else 1
        (base / "numa_node").write_text(f"{node}\n")
        (base / "local_cpulist").write_text(NODE_CPUS[node] + "\n")
    return bdfs


def test_cpulist_roundtrip():
    assert A.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert A.format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    assert A.parse_cpulist("") == []


@pytest.mark.parametrize("cores_per_rank", [14, None])
def test_eight_local_ranks_two_numa_nodes(tmp_path, cores_per_rank):
    bdfs = _fake_sysfs(tmp_path)
    allowed = list(range(224))
    sets = []
    for r in range(8):
        rec = A.bind_to_device(r, r, 8, cores_per_rank=cores_per_rank, sysfs=str(tmp_path),
                               bdf_of=bdfs.get, apply=False, allowed=allowed)
        assert rec["numa_node"] == (0 if r < 4 else 1) and rec["device_bdf"] == bdfs[r]
        cpus = A.parse_cpulist(rec["planned"])
        node_cpus = set(A.parse_cpulist(NODE_CPUS[rec["numa_node"]]))
        assert set(cpus) <= node_cpus                    # GPU-local cores only
        assert len(cpus) == (cores_per_rank or 112 // 4)
        sets.append(set(cpus))
    for i in range(8):                                   # disjoint across local ranks
        for j in range(i + 1, 8):
            assert not sets[i] & sets[j], (i, j)


def test_process_mask_is_respected_and_missing_sysfs_is_reported(tmp_path):
    bdfs = _fake_sysfs(tmp_path)
    rec = A.bind_to_device(5, 5, 8, cores_per_rank=14, sysfs=str(tmp_path), bdf_of=bdfs.get,
                           apply=False, allowed=list(range(8)))      # no node-1 CPU allowed
    assert rec["bound"] is False and "allowed" in rec["reason"]
    rec = A.bind_to_device(0, 0, 1, sysfs=str(tmp_path / "nope"), bdf_of=bdfs.get, apply=False,
                           allowed=list(range(224)))
    assert rec["bound"] is False and "unknown" in rec["reason"]


def test_binding_disabled_by_env(monkeypatch):
    monkeypatch.setenv("DLBB_BIND", "0")
    assert A.bind_to_device(0, 0, 1)["reason"] == "DLBB_BIND=0"


def test_local_env_launchers(monkeypatch):
    from distributed_llm_backend_benchmark_amd.parallel.comm import local_env

    for v in ("LOCAL_RANK", "LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK",
              "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALRANKID", "MPI_LOCALNRANKS",
              "SLURM_LOCALID", "SLURM_NTASKS_PER_NODE"):
        monkeypatch.delenv(v, raising=False)
    assert local_env(9) == (9, 0)
    monkeypatch.setenv("OMPI_COMM_WORLD_LOCAL_RANK", "1")
    monkeypatch.setenv("OMPI_COMM_WORLD_LOCAL_SIZE", "8")
    assert local_env(9) == (1, 8)
    monkeypatch.delenv("OMPI_COMM_WORLD_LOCAL_RANK")
    monkeypatch.delenv("OMPI_COMM_WORLD_LOCAL_SIZE")
    monkeypatch.setenv("SLURM_LOCALID", "3")
    monkeypatch.setenv("SLURM_NTASKS_PER_NODE", "8(x2)")
    assert local_env(11) == (3, 8)
