"""Launch planning for one-process-per-GPU runs (bench.py, train.py).

The reference is single-process, single-device (``/root/reference/train.py:28-29``). Here a run
of N ranks is N processes, rank r on device r, over RCCL (``torch.distributed`` backend
``nccl``). Two ways in:

* under a launcher (``python -m torch.distributed.run --nproc-per-node N ...``): WORLD_SIZE /
  RANK / LOCAL_RANK come from the environment; a ``--gpus`` that disagrees with WORLD_SIZE is an
  error (never silently measure a different width);
* standalone (``python bench.py --gpus N``, WORLD_SIZE unset): the parent starts the N ranks as
  ONE child ``torch.distributed.run`` process and exits with its code. The parent never
  initialises the GPU (``torch.cuda.device_count()`` does not, on ROCm): it checks the device
  count and spawns -- no ``exec`` from a process that touched the device.

``MACBF_DP_BACKEND=gloo`` is the rehearsal mode: several ranks may share one device (RCCL places
exactly one rank per device; gloo does not care). Every other backend requires one distinct
device per rank.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from dataclasses import dataclass


class LaunchError(SystemExit):
    """A launch that cannot measure what was asked (exits non-zero with the message)."""

    def __init__(self, msg: str):
        super().__init__(f"launch error: {msg}")


@dataclass
class Plan:
    action: str            # "run" (this process is a rank) | "spawn" (start `ranks` children)
    ranks: int             # world size of the run
    rank: int = 0
    local_rank: int = 0
    share_devices: bool = False    # gloo rehearsal: ranks may share a device


def rehearsal_backend(environ=None) -> bool:
    environ = os.environ if environ is None else environ
    return (environ.get("MACBF_DP_BACKEND") or "").lower() == "gloo"


def plan(gpus: int | None, environ=None, device_count: int = 0, device: str = "hip") -> Plan:
    """Decide what this process does for a run of ``gpus`` ranks (None: whatever the launcher set).

    device "cpu": ranks run on the host (gloo); no device checks."""
    environ = os.environ if environ is None else environ
    share = rehearsal_backend(environ) or device == "cpu"
    ws = environ.get("WORLD_SIZE")
    if gpus is not None and gpus < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {gpus})")
    if ws is None:
        n = 1 if gpus is None else gpus
        if device != "cpu" and device_count < 1:
            raise LaunchError("no HIP device visible")
        if device != "cpu" and not share and device_count < n:
            raise LaunchError(f"--gpus {n} needs {n} HIP devices (one RCCL rank per device); "
                              f"{device_count} visible. Use MACBF_DP_BACKEND=gloo to rehearse "
                              f"{n} ranks on fewer devices.")
        return Plan("spawn" if n > 1 else "run", n, share_devices=share)
    world = int(ws)
    rank = int(environ.get("RANK", "0"))
    local = int(environ.get("LOCAL_RANK", str(rank)))
    if gpus is not None and gpus != world:
        raise LaunchError(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    if not (0 <= rank < world) or local < 0:
        raise LaunchError(f"bad RANK={rank} / LOCAL_RANK={local} for WORLD_SIZE={world}")
    if device != "cpu":
        if device_count < 1:
            raise LaunchError("no HIP device visible")
        if not share and local >= device_count:
            raise LaunchError(f"LOCAL_RANK {local} has no device of its own ({device_count} visible); "
                              f"RCCL needs one device per rank")
    return Plan("run", world, rank=rank, local_rank=local, share_devices=share)


def device_index(p: Plan, device_count: int) -> int:
    """Rank -> device: local rank r binds device r (rehearsal: round-robin over the devices)."""
    if p.share_devices:
        return p.local_rank % max(device_count, 1)
    return p.local_rank


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_cmd(script: str, argv: list[str], ranks: int, port: int | None = None) -> list[str]:
    """The child launcher command: one torch.distributed.run process starting `ranks` ranks of
    `script` with the same arguments (the ranks then see WORLD_SIZE and run)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
            "--master-addr=127.0.0.1", f"--master-port={port or free_port()}", script, *argv]


def spawn(script: str, argv: list[str], ranks: int) -> int:
    """Start the ranks as a child process group and return its exit code (the caller exits
    with it)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this host driver
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(spawn_cmd(script, argv, ranks), env=env)
