"""Per-rank host-thread binding to the GPU's NUMA node.

The reference pins every rank to cores: ``launch_openmpi.sh:19-23`` (``mpirun --bind-to core
--map-by socket:PE=14``, with ``parallelism.cores_per_rank: 14`` in
``config/baseline_config.yaml:16-18``) and ``collectives/3d/launch_dsccl.sh:69-74``
(``deepspeed --bind_cores_to_rank --bind_core_list`` from the ``rank cores threads`` table
``collectives/3d/config_8.txt``). On an 8 x MI355X node the host threads that issue kernels and
RCCL calls belong on the socket the rank's GPU hangs off: a rank issuing from the far socket pays
cross-socket latency on every doorbell / event poll, which shows up in small-message latency and
in the (partly host-bound) eager TP forward.

Done in-process at ``init_distributed`` — no ``numactl`` relaunch and no exec after GPU init:

1. the device's PCI address from its properties (``pci_domain_id:pci_bus_id:pci_device_id``),
2. ``/sys/bus/pci/devices/<bdf>/numa_node`` and ``local_cpulist``,
3. the local ranks whose GPUs share that CPU list split it into disjoint slices
   (``cores_per_rank`` each when given, else an even share), intersected with the CPUs this
   process may use (cgroup / launcher mask) — unless the launcher already pinned this rank to
   part of the list (its mask differs from its peers'), which is then kept as is;
4. the mask is applied to EVERY thread of the process (``/proc/self/task``: the HIP runtime,
   RCCL proxy, process-group watchdog and OpenMP threads created before this point, not only
   the caller — Linux ``sched_setaffinity(0, …)`` binds one thread), as the reference's
   launchers bind the whole process; threads created later inherit it;
5. with an explicit ``cores_per_rank``, ``torch.set_num_threads`` / ``OMP_NUM_THREADS`` /
   ``MKL_NUM_THREADS`` follow the slice (otherwise the launcher's thread settings stand).

``DLBB_BIND=0`` disables it. The applied binding is recorded in result JSONs.
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence


def parse_cpulist(text: str) -> List[int]:
    """Kernel cpulist syntax (``"0-13,56-69"``, ``"3"``, ``""``) -> sorted CPU ids."""
    out = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.update(range(int(lo), int(hi) + 1))
        else:
            out.add(int(part))
    return sorted(out)


def format_cpulist(cpus: Sequence[int]) -> str:
    """Sorted CPU ids -> compact cpulist (``[0,1,2,5]`` -> ``"0-2,5"``)."""
    cpus = sorted(set(int(c) for c in cpus))
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def device_bdf(index: int) -> Optional[str]:
    """PCI address ``dddd:bb:dd.0`` of HIP device ``index`` (None when unknown)."""
    import torch

    try:
        p = torch.cuda.get_device_properties(index)
        dom, bus, dev = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id",
                                                       "pci_device_id"))
    except Exception:  # noqa: BLE001 - binding is best effort
        return None
    if bus is None or dev is None:
        return None
    return f"{int(dom or 0):04x}:{int(bus):02x}:{int(dev):02x}.0"


def numa_of(bdf: str, sysfs: str = "/sys") -> Dict:
    """``{"numa_node": n, "cpus": [...]}`` of a PCI device from sysfs (empty cpus: unknown)."""
    base = os.path.join(sysfs, "bus", "pci", "devices", bdf)
    node, cpus = -1, []
    try:
        with open(os.path.join(base, "numa_node")) as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(base, "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
    except (OSError, ValueError):
        pass
    if not cpus and node >= 0:       # some kernels expose only the node: use the node's list
        try:
            with open(os.path.join(sysfs, "devices", "system", "node", f"node{node}",
                                   "cpulist")) as f:
                cpus = parse_cpulist(f.read())
        except (OSError, ValueError):
            pass
    return {"numa_node": node, "cpus": cpus}


def plan(local_rank: int, local_cpus: Sequence[Sequence[int]],
         cores_per_rank: Optional[int] = None,
         allowed: Optional[Sequence[int]] = None,
         peers_allowed: Optional[Sequence[Optional[Sequence[int]]]] = None) -> List[int]:
    """The CPU set of ``local_rank`` given every local rank's GPU-local CPU list
    (``local_cpus[r]``). Ranks with the same list share it in disjoint slices, in local-rank
    order: ``cores_per_rank`` cores each when given (reference ``--map-by socket:PE=14``), else
    an even split. ``allowed`` (the process's current mask) is applied first. Falls back to the
    whole (allowed) list when the slice would be empty.

    Launcher-pinned ranks: without ``cores_per_rank``, when ``allowed`` already
    leaves out part of the GPU-local list, the launcher (``mpirun --map-by socket:PE=14``,
    Slurm) or a cgroup placed this rank — its mask is kept as is instead of being cut into a
    1/peers slice of itself. The even split still applies when ``peers_allowed`` (every local
    rank's mask) shows all ranks sharing the list were given the SAME mask (nothing placed them
    apart)."""
    full = list(local_cpus[local_rank])
    mine = full
    if allowed is not None:
        allow = set(allowed)
        mine = [c for c in mine if c in allow]
    if not mine:
        return []
    peers = [r for r in range(len(local_cpus)) if list(local_cpus[r]) == full]
    if cores_per_rank is None and len(mine) < len(full) and len(peers) > 1:
        same = peers_allowed is not None and all(
            peers_allowed[r] is not None and sorted(peers_allowed[r]) == sorted(allowed)
            for r in peers if r < len(peers_allowed))
        if not same:
            return mine
    slot = peers.index(local_rank)
    n = int(cores_per_rank) if cores_per_rank else max(1, len(mine) // len(peers))
    chunk = mine[slot * n:(slot + 1) * n]
    return chunk if chunk else mine


def _local_device_indices(local_world: int, ndev: int) -> List[int]:
    return [r % max(1, ndev) for r in range(local_world)]


def thread_ids() -> List[int]:
    """Every thread (task) id of this process (``/proc/self/task``); empty where unavailable."""
    try:
        return sorted(int(t) for t in os.listdir("/proc/self/task"))
    except (OSError, ValueError):
        return []


def apply_to_all_threads(cpus: Sequence[int]) -> Dict:
    """Set the affinity of EVERY thread of the process to ``cpus`` (threads that exit meanwhile
    are skipped) and read each back: ``{"threads": n, "threads_bound": k, "threads_outside":
    [tids still outside]}``. Also binds the calling thread first, so threads it creates later
    inherit the mask."""
    want = set(cpus)
    os.sched_setaffinity(0, cpus)
    bound, outside, seen = 0, [], 0
    for tid in thread_ids():
        try:
            os.sched_setaffinity(tid, cpus)
            got = os.sched_getaffinity(tid)
        except OSError:          # the thread exited between listing and binding
            continue
        seen += 1
        if set(got) <= want:
            bound += 1
        else:
            outside.append(tid)
    return {"threads": seen, "threads_bound": bound, "threads_outside": outside}


def bind_to_device(device_index: int, local_rank: int, local_world: int,
                   cores_per_rank: Optional[int] = None, sysfs: str = "/sys",
                   bdf_of=None, apply: bool = True,
                   allowed: Optional[Sequence[int]] = None,
                   peers_allowed: Optional[Sequence[Optional[Sequence[int]]]] = None) -> Dict:
    """Bind this process (every thread) to its GPU's NUMA-local cores (see module doc). Returns
    the record written into result JSONs; never raises (``{"bound": False, "reason": ...}``).
    ``peers_allowed``: every local rank's CPU mask before binding (gathered at init), for the
    launcher-pinned rule of :func:`plan`. ``bdf_of`` / ``apply=False`` / ``allowed``: test
    hooks (a fake device -> PCI map, plan without binding, a fake process mask)."""
    rec: Dict = {"bound": False, "local_rank": local_rank, "device": device_index}
    bdf_of = bdf_of or device_bdf
    if os.environ.get("DLBB_BIND", "1") == "0":
        rec["reason"] = "DLBB_BIND=0"
        return rec
    if not hasattr(os, "sched_setaffinity"):
        rec["reason"] = "no sched_setaffinity"
        return rec
    import torch

    try:
        ndev = torch.cuda.device_count() if bdf_of is device_bdf else local_world
    except Exception:  # noqa: BLE001
        ndev = 0
    if ndev <= 1 and local_world > 1:
        # one GPU visible per process (HIP_VISIBLE_DEVICES per rank): the peers' GPUs are not
        # visible here, so this rank takes the first slice of its own GPU's list
        devs, local_rank = [device_index], 0
    else:
        devs = _local_device_indices(max(local_world, local_rank + 1), ndev)
        devs[local_rank] = device_index
    infos = {}
    for d in set(devs):
        bdf = bdf_of(d)
        infos[d] = dict(numa_of(bdf, sysfs), bdf=bdf) if bdf else {"numa_node": -1, "cpus": [],
                                                                   "bdf": None}
    me = infos[device_index]
    rec.update(numa_node=me["numa_node"], device_bdf=me["bdf"])
    if not me["cpus"]:
        rec["reason"] = "GPU-local CPU list unknown (no sysfs entry)"
        return rec
    if allowed is None:
        allowed = sorted(os.sched_getaffinity(0))
    if peers_allowed is not None and len(peers_allowed) != len(devs):
        peers_allowed = None                  # one GPU per process: peers not visible here
    cpus = plan(local_rank, [infos[d]["cpus"] for d in devs], cores_per_rank, allowed,
                peers_allowed)
    if not cpus:
        rec["reason"] = "no GPU-local CPU in this process's allowed set"
        return rec
    if not apply:
        return dict(rec, planned=format_cpulist(cpus), ncpus=len(cpus))
    try:
        threads = apply_to_all_threads(cpus)
    except OSError as e:
        rec["reason"] = f"sched_setaffinity: {e}"
        return rec
    n = len(cpus)
    if cores_per_rank:
        # an explicit per-rank core budget (reference: OMP/MKL threads = cores per rank,
        # config/baseline_config.yaml system section): intra-op threads follow it; without one
        # the launcher's thread settings are left alone
        os.environ["OMP_NUM_THREADS"] = os.environ["MKL_NUM_THREADS"] = str(n)
        try:
            torch.set_num_threads(n)
        except RuntimeError:
            pass
    rec.update(bound=True, cpus=format_cpulist(cpus), ncpus=n,
               cores_per_rank=cores_per_rank, **threads)
    return rec


def current() -> Dict:
    """This process's CPU mask — the union over its threads, and how many threads it has (for
    result JSONs)."""
    try:
        cpus = set(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return {}
    tids = thread_ids()
    for tid in tids:
        try:
            cpus |= set(os.sched_getaffinity(tid))
        except OSError:
            pass
    return {"cpus": format_cpulist(sorted(cpus)), "ncpus": len(cpus), "threads": len(tids)}
