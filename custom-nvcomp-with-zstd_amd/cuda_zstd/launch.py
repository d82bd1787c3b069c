"""One process per GPU for the sharded batch path.

``bench.py --gpus N`` must run N ranks whether or not the caller wrapped it in torchrun.
When the rank environment (``WORLD_SIZE``) is absent, the parent process starts
``python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1``
over the same script and arguments as a CHILD process and returns its exit code: the
parent never touches the GPU (it only counts devices, which does not initialise HIP on
this image) and never ``exec``s, so nothing replaces a process that holds a GPU context.
Each child rank then finds RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in its environment
and opens its process group (RCCL on the GPU, gloo in the CPU tests).

The reference has no multi-GPU path (/root/reference/README.md:1637,1648); this is the
north star's C4 split, not a restatement of reference code.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Mapping, Sequence


def rank_env_present(env: Mapping[str, str] | None = None) -> bool:
    """True when this process is already one rank of a launched job (torchrun, the driver)."""
    env = os.environ if env is None else env
    return "WORLD_SIZE" in env


def rank_env(env: Mapping[str, str] | None = None):
    """(rank, local_rank, world) from the launcher's environment; (0, 0, 1) without one."""
    env = os.environ if env is None else env
    return int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0")), int(env.get("WORLD_SIZE", "1"))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_command(nproc: int, script: str, argv: Sequence[str], port: int) -> list:
    """The torchrun command line that runs `script argv` as `nproc` ranks on this node."""
    if nproc < 1:
        raise ValueError(f"nproc must be >= 1, got {nproc}")
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(port), script, *argv]


def spawn_ranks(nproc: int, script: str, argv: Sequence[str], port: int | None = None,
                env: Mapping[str, str] | None = None, timeout: float | None = None) -> int:
    """Run `script argv` as `nproc` ranks (children of this process, stdout/stderr inherited so
    rank 0's line reaches the caller) and return their exit code.  The environment keeps
    HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC, which RCCL needs on this driver)."""
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e.setdefault("MASTER_ADDR", "127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    cmd = launch_command(nproc, script, argv, port or free_port())
    return subprocess.run(cmd, env=e, timeout=timeout).returncode


def visible_gpus() -> int:
    """GPUs this process may use, counted without initialising HIP."""
    import torch

    return torch.cuda.device_count()
