"""Race-free process launchers for the multi-process tests.

The round-5 launchers picked a port by binding port 0, closing the socket and handing the
number to torchrun; any other socket on the box could take it in between, and the driver's GPU
suite stopped on ``EADDRINUSE`` after 96 tests. Two launch forms replace that:

* ``run_torchrun``: ``torchrun --standalone`` -- the agent binds its rendezvous store and the
  shared worker store on port 0 itself (atomic), the workers join the agent's store as clients
  (``TORCHELASTIC_USE_AGENT_STORE=True``). A caller may still pass an explicit ``port`` (the
  driver's static form); if that launch fails on ``EADDRINUSE`` the launcher -- a process that
  never touched a GPU -- is started again as a fresh child in the standalone form.
* ``hold_store``: for ``torch.multiprocessing`` workers (``mp_utils``) the PARENT binds a
  ``TCPStore`` on port 0 and keeps it for the workers' lifetime; the workers' ``env://``
  rendezvous then connects to it as clients only (agent-store mode), so no worker binds a port.
"""

import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_IN_USE = ("EADDRINUSE", "address already in use", "Address already in use")


def addr_in_use(text: str) -> bool:
    return any(s in (text or "") for s in _IN_USE)


def torchrun_cmd(nproc: int, port=None):
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
            str(nproc)]
    if port is None:
        return base + ["--standalone", "--local-addr", "127.0.0.1"]
    return base + ["--master-addr", "127.0.0.1", "--master-port", str(port)]


def run_torchrun(nproc: int, args, timeout: float, env=None, cwd=REPO, port=None,
                 attempts: int = 3):
    """Run ``torchrun <args>`` with ``nproc`` workers; returns the CompletedProcess of the last
    attempt. Only an address-in-use failure is retried (fresh launcher, standalone form)."""
    env = dict(os.environ if env is None else env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = None
    for i in range(attempts):
        out = subprocess.run(torchrun_cmd(nproc, port) + list(args), capture_output=True,
                             text=True, timeout=timeout, cwd=cwd, env=env)
        if out.returncode == 0 or i == attempts - 1 or not addr_in_use(out.stderr + out.stdout):
            return out
        port = None
    return out


def hold_store(world: int):
    """A TCPStore server owned by the calling process, bound on port 0 (atomic). Keep the
    returned object alive while the workers run; pass ``store.port`` to them."""
    import datetime

    import torch.distributed as dist

    return dist.TCPStore("127.0.0.1", 0, world, is_master=True, wait_for_workers=False,
                         timeout=datetime.timedelta(seconds=300))
