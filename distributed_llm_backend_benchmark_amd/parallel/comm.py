"""Process-group layer: ONE ``torch.distributed`` group per job.

Replaces the reference's four CPU launch/backends (mpi4py ``COMM_WORLD``
``run_mpi.py:29-43``, ``deepspeed.init_distributed(dist_backend=...)``
``collectives/1d/dsccl.py:47-57``) with:

* ``rccl`` — ``torch.distributed`` backend ``"nccl"``, which on ROCm is RCCL over xGMI.
  One process per GPU; ``LOCAL_RANK`` selects the device.
* ``gloo`` — CPU plumbing backend (BASELINE config 1, tests).

Rendezvous comes from the launcher env (``torchrun``: RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/
MASTER_PORT). Without it a single-process world is created on 127.0.0.1. A process-group
timeout makes a hung collective fail fast instead of eating the job's time limit
(SURVEY §5.3).
"""

from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass, field
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist

BACKEND_ALIASES = {"rccl": "nccl", "nccl": "nccl", "gloo": "gloo", "cpu": "gloo"}


def resolve_backend(name: str = "auto") -> str:
    name = (name or "auto").lower()
    if name == "auto":
        return "nccl" if torch.cuda.is_available() else "gloo"
    if name not in BACKEND_ALIASES:
        raise ValueError(f"unknown backend {name!r}; expected rccl|gloo|auto")
    return BACKEND_ALIASES[name]


@dataclass
class Comm:
    """Thin handle over the default process group plus the rank's device."""

    rank: int
    world_size: int
    local_rank: int
    backend: str               # torch backend string: "nccl" (RCCL) or "gloo"
    device: torch.device
    owns_pg: bool = False
    _extra: dict = field(default_factory=dict)

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    @property
    def backend_label(self) -> str:
        return "rccl" if self.backend == "nccl" else self.backend

    @property
    def affinity(self) -> dict:
        """The host-thread binding applied at init (``utils.affinity.bind_to_device``)."""
        from ..utils.affinity import current

        return dict(self._extra.get("affinity") or {"bound": False}, **current())

    def affinity_all_ranks(self) -> List[dict]:
        """Collective: every rank's :attr:`affinity` (result JSONs report them per rank)."""
        return self.all_gather_object(dict(self.affinity, rank=self.rank))

    # ---------------------------------------------------------------- sync helpers
    def barrier(self) -> None:
        if self.world_size == 1:
            if self.is_gpu:
                torch.cuda.synchronize(self.device)
            return
        if self.backend == "nccl":
            dist.barrier(device_ids=[self.device.index])
        else:
            dist.barrier()

    def sync(self) -> None:
        if self.is_gpu:
            torch.cuda.synchronize(self.device)

    # ---------------------------------------------------------------- side channel
    def gather_floats(self, values: Sequence[float], dst: int = 0) -> Optional[List[List[float]]]:
        """Gather a per-rank list of floats to ``dst`` as ``[rank][i]``.

        Reference: ``comm.gather(timings)`` (``collectives/1d/openmpi.py:270``) and
        ``dist.gather(float64 tensor)`` (``collectives/1d/dsccl.py:225-232``). Lists may differ
        in length across ranks, so lengths travel first.
        """
        if self.world_size == 1:
            return [list(map(float, values))]
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        n = torch.tensor([len(values)], dtype=torch.int64, device=dev)
        ns = [torch.zeros_like(n) for _ in range(self.world_size)]
        dist.all_gather(ns, n)
        nmax = int(max(int(x.item()) for x in ns))
        buf = torch.zeros(nmax, dtype=torch.float64, device=dev)
        if len(values):
            buf[: len(values)] = torch.tensor(list(values), dtype=torch.float64, device=dev)
        outs = [torch.zeros_like(buf) for _ in range(self.world_size)]
        dist.all_gather(outs, buf)
        if self.rank != dst:
            return None
        return [outs[r][: int(ns[r].item())].cpu().tolist() for r in range(self.world_size)]

    def all_gather_object(self, obj: Any) -> List[Any]:
        if self.world_size == 1:
            return [obj]
        out: List[Any] = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if self.world_size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src)
        return lst[0]

    def allreduce_max(self, x: float) -> float:
        if self.world_size == 1:
            return float(x)
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def cpu_group(self):
        """A gloo group over the same ranks for host-side agreement traffic that must not be
        queued behind (or interleaved with) RCCL kernels on the device; None when the default
        group is already gloo or there is one rank. Creating it is collective: the first call
        must happen at the same point on every rank."""
        if self.world_size == 1 or self.backend == "gloo":
            return None
        g = self._extra.get("cpu_group")
        if g is None:
            # its own (short) timeout: a rank that never reaches an agreement point (a GEMM
            # shape only some ranks tune, a section one rank skipped) fails the job in minutes,
            # not after the default group's 900 s
            secs = float(os.environ.get("DLBB_SIDE_GROUP_TIMEOUT_S", "300"))
            g = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=secs))
            self._extra["cpu_group"] = g
        return g

    def agree_max(self, names: Sequence[str], values: Sequence[float]) -> List[float]:
        """Collective: the element-wise MAX of ``values`` over all ranks, through the host side
        channel (:meth:`cpu_group`). Every rank must pass the same ``names`` in the same order
        (checked: a mismatch raises on every rank instead of mixing candidates)."""
        vals = [float(v) for v in values]
        if self.world_size == 1:
            return vals
        out: List[Any] = [None] * self.world_size
        dist.all_gather_object(out, (list(names), vals), group=self.cpu_group())
        if any(o[0] != list(names) or len(o[1]) != len(vals) for o in out):
            raise RuntimeError(f"agree_max: ranks disagree on the candidates: {[o[0] for o in out]}")
        return [max(o[1][i] for o in out) for i in range(len(vals))]

    def install_tune_agreement(self) -> None:
        """Make the GEMM autotuner's decisions collective (ops.gemm.set_tune_agreement): every
        rank picks the kernel with the smallest rank-max time. Collective (creates the side
        group): call at the same point on every rank, before the first GEMM."""
        if self.world_size == 1:
            return
        from ..ops import gemm

        self.cpu_group()
        gemm.set_tune_agreement(self.agree_max)
        self._extra["tune_agreement"] = True

    def destroy(self) -> None:
        import sys

        if self._extra.pop("tune_agreement", False):
            from ..ops import gemm

            gemm.set_tune_agreement(None)

        native = sys.modules.get(__package__ + ".rccl_native")
        if native is not None:          # our own RCCL communicators go first
            native.close_all()
        if self.owns_pg and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


# (local rank, local world size) variables of the launchers we may run under: torchrun, Open MPI,
# MPICH / Intel MPI (hydra), Slurm
_LOCAL_RANK_VARS = ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID")
_LOCAL_SIZE_VARS = ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS",
                    "SLURM_NTASKS_PER_NODE")


def local_env(rank: int) -> tuple:
    """(local_rank, local_world or 0 when no launcher says) from the launcher environment."""
    lr = next((os.environ[v] for v in _LOCAL_RANK_VARS if os.environ.get(v)), None)
    lw = next((os.environ[v] for v in _LOCAL_SIZE_VARS if os.environ.get(v)), None)
    try:
        lw = int(str(lw).split("(")[0].split(",")[0]) if lw is not None else 0  # "8(x2)" slurm
    except ValueError:
        lw = 0
    return (int(lr) if lr is not None else rank), lw


def init_distributed(backend: str = "auto", timeout_s: float = 600.0,
                     device: Optional[str] = None,
                     cores_per_rank: Optional[int] = None) -> Comm:
    """Initialise (or attach to) the default process group.

    ``backend``: ``rccl`` | ``nccl`` | ``gloo`` | ``auto``. ``device`` overrides the device
    choice (``"cpu"`` forces CPU tensors even on a GPU box, e.g. gloo plumbing runs).
    On a HIP device the process's host threads are bound to the GPU's NUMA-local cores
    (``utils.affinity``; ``cores_per_rank`` = the reference's ``parallelism.cores_per_rank``,
    ``launch_openmpi.sh:19-23``); the record is ``comm.affinity``.
    """
    be = resolve_backend(backend)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank, local_world = local_env(rank)

    if be == "nccl":
        if not torch.cuda.is_available():
            raise RuntimeError("backend rccl requested but no HIP device is visible")
        ndev = torch.cuda.device_count()
        if local_world == 0 and world > ndev > 1 and local_rank >= ndev:
            import warnings

            # no launcher variable gives the local world size: if this is ONE node, two ranks
            # now share a GPU and RCCL fails late (duplicate device); on several nodes it is fine
            warnings.warn(f"local rank {local_rank} (no LOCAL_WORLD_SIZE / OMPI / Slurm local "
                          f"size set) mapped to device {local_rank % ndev} of {ndev} by modulo: "
                          "correct across nodes, a duplicate-GPU error if all ranks share one "
                          "node", RuntimeWarning, stacklevel=2)
        if local_world > ndev:
            # RCCL refuses two ranks on one GPU only late (duplicate-device error at the first
            # collective); fail at init with the reason instead
            raise RuntimeError(
                f"{local_world} local ranks but only {ndev} visible HIP device(s): RCCL needs "
                f"one GPU per rank (launch at most {ndev} ranks per node, or use backend gloo "
                f"with device='cuda' to share a GPU for rehearsals)")
        # launchers that set no LOCAL_RANK (mpirun / srun: LOCAL_RANK defaults to the global
        # rank) or expose one GPU per process (ndev == 1) map by modulo
        dev_index = local_rank % ndev
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    else:
        dev = torch.device(device or "cpu")
        if dev.type == "cuda":
            torch.cuda.set_device(local_rank % torch.cuda.device_count())
            dev = torch.device("cuda", torch.cuda.current_device())

    owns = False
    if not dist.is_initialized():
        kwargs = dict(backend=be, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if "WORLD_SIZE" not in os.environ:
            # standalone single process: an in-process store, so no port is bound at all (a
            # loopback port picked in advance can be taken by another process before the bind)
            kwargs["store"] = dist.HashStore()
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                raise RuntimeError("MASTER_PORT must be set when WORLD_SIZE is set")
        eager = be == "nccl" and os.environ.get("DLBB_RCCL_EAGER_INIT", "0") == "1"
        if eager:
            kwargs["device_id"] = dev  # eager RCCL communicator init, fixed device binding
        dist.init_process_group(**kwargs)
        owns = True
        if be == "nccl" and not eager:
            # Lazy communicator creation, forced now by one tiny all-reduce on the bound device.
            # The eager path (init_process_group(device_id=...)) leaves this process in a state
            # where kernels on two streams stop running concurrently: the overlapped TP forward
            # (one compute + one comm stream) measured 28.6 ms after an eager world-1 init vs
            # 17.6 ms after a lazy one, same code (tools/diag/tp_overlap_probe.py --pg-eager,
            # profiles/r03_tp/overlap_probe); DLBB_RCCL_EAGER_INIT=1 restores it for A/B.
            t = torch.zeros(1, device=dev)
            dist.all_reduce(t)
            torch.cuda.synchronize(dev)
    else:
        rank, world = dist.get_rank(), dist.get_world_size()
    comm = Comm(rank=rank, world_size=world, local_rank=local_rank, backend=be,
                device=dev, owns_pg=owns)
    if dev.type == "cuda":
        from ..utils.affinity import bind_to_device

        lw = local_world or min(world, 64)
        comm._extra["affinity"] = bind_to_device(dev.index, local_rank, lw,
                                                 cores_per_rank=cores_per_rank,
                                                 peers_allowed=_local_masks(comm, lw))
    return comm


def _local_masks(comm: "Comm", local_world: int):
    """Every local rank's CPU mask before binding (host name + local rank over the process
    group; collective), for the launcher-pinned rule of ``utils.affinity.plan``; None at one
    rank or when unavailable."""
    if comm.world_size == 1 or not hasattr(os, "sched_getaffinity"):
        return None

    host = socket.gethostname()
    mine = (host, comm.local_rank, sorted(os.sched_getaffinity(0)))
    try:
        allv = comm.all_gather_object(mine)
    except RuntimeError:
        return None
    masks = {lr: m for h, lr, m in allv if h == host}
    return [masks.get(r) for r in range(local_world)]
