"""One process per GPU for ``bench.py --gpus N``.

When a script is started with ``--gpus N > 1`` outside a ``torch.distributed.run`` launch
(no ``WORLD_SIZE`` in the environment), ``relaunch`` starts
``python -m torch.distributed.run --nproc-per-node N`` over the same script and arguments as
a CHILD process, streams its output through, and returns its exit code.  It must run
before anything touches the GPU: the parent never initialises HIP (it only counts devices,
which does not), and it never replaces itself with the launcher (no exec).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(script: str, argv: list[str], n: int, port: int) -> list[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
            script, *argv]


def visible_gpus() -> int:
    """GPUs this process may use, without initialising HIP (torch.cuda.device_count reads
    the visible-device list; it does not create a context on this image)."""
    import torch
    return torch.cuda.device_count()


def needs_launch(n: int) -> bool:
    return n > 1 and "WORLD_SIZE" not in os.environ


def relaunch(script: str, argv: list[str], n: int, check_gpus: bool = True) -> int:
    """Run `script argv` as n ranks under torch.distributed.run; returns the exit code."""
    if check_gpus:
        have = visible_gpus()
        if have < n:
            raise SystemExit(f"--gpus {n} asked for {n} ranks but only {have} GPU(s) are "
                             "visible to this process")
    cmd = launcher_cmd(os.path.abspath(script), argv, n, free_port())
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on these hosts
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.run(cmd, env=env)
    return proc.returncode
