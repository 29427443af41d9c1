"""One process per GPU behind a script's own `--gpus N` flag.

`python bench.py --gpus 8` must measure eight ranks, not one. Two ways in:
* under `torch.distributed.run` (the driver's form) WORLD_SIZE is already set: the process is a
  rank; WORLD_SIZE must equal --gpus, or the run is refused;
* started plainly with N > 1: this process becomes a launcher. It never touches the GPU (no HIP
  call, no torch.cuda.is_available(); only torch.cuda.device_count(), which does not initialise
  the runtime on this image), starts N fresh child processes of the same script with RANK,
  LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE and MASTER_ADDR / MASTER_PORT set, waits for them,
  ends the rest when one fails, and exits with the first failing child's code. Rank 0 inherits
  stdout and the other ranks write to stderr, so rank 0's one JSON line is what stdout carries.

The reference has no multi-GPU path (/root/reference/inference.py:3 pins CUDA_VISIBLE_DEVICES=0).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional

RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


class LaunchError(SystemExit):
    """A refused launch: the message goes to stderr and the exit status is 2."""

    def __init__(self, msg: str):
        print(f"[launch] {msg}", file=sys.stderr, flush=True)
        super().__init__(2)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    """GPUs this process could use, counted without initialising the HIP runtime."""
    import torch
    return int(torch.cuda.device_count())


def role(nproc: Optional[int]) -> str:
    """'rank' when the environment already makes this process one rank of a job (or nproc == 1),
    'launcher' when it must start nproc ranks itself. nproc None (--gpus not given): the environment's
    WORLD_SIZE when set (plain `torch.distributed.run --nproc-per-node N script`), else 1. An explicit
    nproc that disagrees with WORLD_SIZE is refused."""
    ws = os.environ.get("WORLD_SIZE")
    if nproc is None:
        return "rank"
    if nproc < 1:
        raise LaunchError(f"--gpus must be >= 1, got {nproc}")
    if ws is not None:
        if int(ws) != nproc:
            raise LaunchError(f"WORLD_SIZE={ws} in the environment disagrees with --gpus {nproc}")
        return "rank"
    return "rank" if nproc == 1 else "launcher"


def spawn(nproc: int, script: str, argv: List[str], *, require_gpus: bool = True,
          poll_s: float = 0.2, env_extra: Optional[dict] = None) -> int:
    """Start nproc ranks of `script argv` on this node and wait; returns the job's exit status
    (0 when every rank exits 0, else the first failing rank's status)."""
    # RDEIC_LAUNCH_SHARE_GPU=1 (rehearsal on a one-GPU box only): ranks share the visible GPUs
    # round-robin and talk over gloo, since RCCL refuses two ranks on one device
    share = os.environ.get("RDEIC_LAUNCH_SHARE_GPU") == "1"
    have = visible_gpus() if (require_gpus or share) else nproc
    if require_gpus and have < nproc and not (share and have >= 1):
        raise LaunchError(f"--gpus {nproc} needs {nproc} visible GPUs, this node shows {have}; "
                          f"one process per GPU, no oversubscription")
    port = _free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r % have if share else r), WORLD_SIZE=str(nproc),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0")
        if share:
            env["RDEIC_DIST_BACKEND"] = "gloo"
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
        if env_extra:
            env.update(env_extra)
        # own process group per rank: a failing job is ended by pgid, never by pattern
        # only rank 0 writes the launcher's stdout (its one JSON line); the other ranks' stdout goes to stderr
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr, start_new_session=True))
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            failed = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if failed:
                r, c = failed[0]
                print(f"[launch] rank {r} exited with status {c}; ending the other ranks", file=sys.stderr,
                      flush=True)
                status = c if c > 0 else 128 - c
                break
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
    except KeyboardInterrupt:
        status = 130
    for p in procs:  # end the survivors of a failed job
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + 20
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
    return status


def maybe_launch(nproc: Optional[int], script: str, argv: Optional[List[str]] = None, **kw) -> None:
    """Call first thing in a `--gpus N` script, before anything touches the GPU: returns when this
    process is a rank; otherwise runs the job as its launcher and exits with the job's status."""
    if role(nproc) == "rank":
        return
    raise SystemExit(spawn(nproc, os.path.abspath(script), sys.argv[1:] if argv is None else argv, **kw))
