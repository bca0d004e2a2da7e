"""Single-node launcher: one process per GPU, the environment contract of
`python -m oneflow.distributed.launch` (reference python/oneflow/distributed/launch.py:103-140):
every child gets MASTER_ADDR / MASTER_PORT / WORLD_SIZE / RANK / LOCAL_RANK and runs the same
script with the same arguments.

Used by bench.py when it is asked for N > 1 GPUs without a launcher around it, so that
`python bench.py --gpus 8` runs 8 ranks instead of silently running one.  The parent never
touches the GPU: it only starts the children and returns the first failing exit code (the
others are terminated, as the reference's sigkill_handler does for the whole group).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def rank_env(base: dict, world: int, rank: int, addr: str, port: int) -> dict:
    """The per-rank environment (launch.py:105-109, 138-140)."""
    env = dict(base)
    env.update(MASTER_ADDR=addr, MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
               LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    return env


def spawn_local_ranks(nproc: int, argv: list, master_addr: str = "127.0.0.1",
                      master_port: int | None = None, env: dict | None = None,
                      timeout: float | None = None) -> int:
    """Runs `python -u <argv...>` as `nproc` ranks on this node; returns 0 when every rank exits
    0, else the first non-zero exit code seen (the remaining ranks are terminated)."""
    if nproc < 1:
        raise ValueError(f"spawn_local_ranks: nproc={nproc}")
    port = master_port or free_port(master_addr)
    base = dict(os.environ if env is None else env)
    procs = [subprocess.Popen([sys.executable, "-u", *argv],
                              env=rank_env(base, nproc, r, master_addr, port))
             for r in range(nproc)]
    t0 = time.monotonic()
    rc = 0
    try:
        alive = list(procs)
        while alive:
            for p in list(alive):
                code = p.poll()
                if code is None:
                    continue
                alive.remove(p)
                if code < 0:  # killed by a signal: the shell's 128 + signo
                    code = 128 - code
                if code != 0 and rc == 0:
                    rc = code
            if rc != 0 or (timeout is not None and time.monotonic() - t0 > timeout):
                if rc == 0:
                    rc = 124  # timeout(1)'s status
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc
