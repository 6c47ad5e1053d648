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


def test_launcher_pinned_mask_is_kept_unless_all_peers_share_it():
    """a rank the launcher already pinned inside its GPU-local list (mpirun
    --map-by socket:PE=14) keeps that mask instead of a 1/peers slice of it; identical masks
    on every peer (nothing placed them apart) are still split evenly."""
    local = [A.parse_cpulist("0-55")] * 4
    pinned = [list(range(14 * r, 14 * r + 14)) for r in range(4)]
    for r in range(4):
        assert A.plan(r, local, allowed=pinned[r], peers_allowed=pinned) == pinned[r]
        assert A.plan(r, local, allowed=pinned[r]) == pinned[r]      # peers unknown: keep
    shared = list(range(0, 40))                                      # cgroup, same for all
    got = [A.plan(r, local, allowed=shared, peers_allowed=[shared] * 4) for r in range(4)]
    assert [len(g) for g in got] == [10] * 4
    assert len(set().union(*map(set, got))) == 40
    full = list(range(224))                                          # unrestricted: split
    assert A.plan(1, local, allowed=full) == list(range(14, 28))


def test_binding_applies_to_every_thread(tmp_path):
    """threads that exist BEFORE bind_to_device (HIP runtime, RCCL proxy,
    PG watchdog in a real run) end up inside the planned set too, not only the caller; the
    original mask is restored afterwards."""
    import threading

    orig = sorted(os.sched_getaffinity(0))
    if len(orig) < 2:
        pytest.skip("needs at least 2 CPUs")
    half = orig[: len(orig) // 2]
    base = tmp_path / "bus" / "pci" / "devices" / "0000:11:00.0"
    base.mkdir(parents=True)
    (base / "numa_node").write_text("0\n")
    (base / "local_cpulist").write_text(A.format_cpulist(half) + "\n")
    stop = threading.Event()
    tids = []
    ready = threading.Barrier(4)

    def worker():
        tids.append(threading.get_native_id())
        ready.wait()
        stop.wait(30)

    ths = [threading.Thread(target=worker, daemon=True) for _ in range(3)]
    for t in ths:
        t.start()
    ready.wait()
    try:
        rec = A.bind_to_device(0, 0, 1, sysfs=str(tmp_path), bdf_of={0: "0000:11:00.0"}.get)
        assert rec["bound"] is True, rec
        planned = set(A.parse_cpulist(rec["cpus"]))
        assert planned == set(half)
        assert rec["threads"] >= 4 and rec["threads_bound"] == rec["threads"]
        assert rec["threads_outside"] == []
        for tid in tids:                                  # created before the binding
            assert set(os.sched_getaffinity(tid)) <= planned, tid
        t_new = threading.Thread(target=lambda: tids.append(-threading.get_native_id()))
        t_new.start()
        t_new.join()
        cur = A.current()
        assert A.parse_cpulist(cur["cpus"]) == sorted(planned)
    finally:
        stop.set()
        for t in ths:
            t.join()
        A.apply_to_all_threads(orig)
    assert sorted(os.sched_getaffinity(0)) == orig
