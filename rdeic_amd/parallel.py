"""Data-parallel codec over the GPUs of one node (one process per GPU, torch.distributed on
RCCL over xGMI). Images are independent units: each rank codes its contiguous shard of the
global batch with no collective on the data path; the only collective is ONE all-gather of the
per-image metric rows at batch end. The reference itself is single-GPU
(inference.py:3 pins CUDA_VISIBLE_DEVICES=0)."""
from __future__ import annotations

import os
from typing import Tuple

import torch
import torch.distributed as dist

METRIC_FIELDS = ("bpp", "bytes", "psnr", "mse", "decode_ok", "rank")


def init_from_env(backend: str = None) -> Tuple[int, int, int]:
    """Returns (rank, world, local_rank); initialises the process group when WORLD_SIZE > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def shard(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, end) of the global batch owned by `rank`."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_metrics(rows: torch.Tensor) -> torch.Tensor:
    """All-gather [B_local, k] fp32 metric rows -> [world * B_local, k] (equal shards)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return rows
    world = dist.get_world_size()
    out = torch.empty((world * rows.shape[0], rows.shape[1]), dtype=rows.dtype, device=rows.device)
    dist.all_gather_into_tensor(out, rows.contiguous())
    return out


def max_over_ranks(value: float, device) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and device.type == "cuda":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
