"""Launcher: one process per GPU (SURVEY §7.1 principle 4).

``python -m deep_vision_amd.launch --nproc 8 <script.py> [args]`` or ``--nproc N`` on any family
entry point: re-runs the command under ``torch.distributed.run`` (rendezvous on 127.0.0.1) as a
*child process* and exits with its status -- the parent never touches the GPU, so nothing is
exec'ed from a GPU-initialised process.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(nproc: int, argv, module: str | None = None) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}"]
    cmd += (["-m", module] if module else []) + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def maybe_spawn(nproc) -> None:
    """Called first thing by the entry points: with ``--nproc N > 1`` outside a torchrun world,
    re-launch this script N times and exit."""
    if not nproc or nproc <= 1 or "WORLD_SIZE" in os.environ:
        return
    argv = list(sys.argv)
    # drop the --nproc flag so the children do not spawn again
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == "--nproc":
            skip = True
            continue
        if a.startswith("--nproc="):
            continue
        out.append(a)
    sys.exit(spawn(nproc, out))


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("-m", "--module", default=None)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    sys.exit(spawn(a.nproc, a.rest, a.module))


if __name__ == "__main__":
    main()
