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

METRIC_FIELDS = ("bpp", "bytes", "psnr", "mse", "ms_ssim", "decode_ok", "rank")


def init_from_env(backend: str = None) -> Tuple[int, int, int]:
    """Returns (rank, world, local_rank); initialises the process group when WORLD_SIZE > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:  # RDEIC_DIST_BACKEND=gloo: launcher rehearsals with several ranks on one GPU
            backend = os.environ.get("RDEIC_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend=backend)
        else:
            # gloo's C++ side prints "[Gloo] Rank i is connected ..." on the process's stdout, which must
            # carry nothing but rank 0's JSON line: route fd 1 to stderr while the mesh connects
            import sys
            sys.stdout.flush()
            saved = os.dup(1)
            try:
                os.dup2(2, 1)
                dist.init_process_group(backend=backend)
                dist.barrier()
            finally:
                os.dup2(saved, 1)
                os.close(saved)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def shard(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, end) of the global batch owned by `rank`."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def _gloo() -> bool:
    return dist.get_backend() == "gloo"


def gather_metrics(rows: torch.Tensor, global_batch: int = None) -> torch.Tensor:
    """All-gather each rank's [B_local, k] fp32 metric rows -> [global_batch, k] in global image
    order. Shards come from shard(global_batch, ...), so they may differ by one row: every rank
    pads to the largest shard, ONE all_gather_into_tensor moves [world, B_max, k], and the padding
    is dropped by the known shard sizes (no second collective for the sizes)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return rows
    world, rank = dist.get_world_size(), dist.get_rank()
    if global_batch is None:
        global_batch = world * rows.shape[0]
    sizes = [shard(global_batch, r, world) for r in range(world)]
    if rows.shape[0] != sizes[rank][1] - sizes[rank][0]:
        raise ValueError(f"rank {rank} holds {rows.shape[0]} rows, its shard of {global_batch} is {sizes[rank]}")
    bmax = max(e - s for s, e in sizes)
    dev = rows.device
    if _gloo():  # gloo collectives on host tensors (RCCL takes the device tensor as is)
        rows = rows.cpu()
    send = rows.new_zeros((bmax, rows.shape[1]))
    send[: rows.shape[0]] = rows
    out = torch.empty((world * bmax, rows.shape[1]), dtype=rows.dtype, device=rows.device)
    dist.all_gather_into_tensor(out, send)
    out = out.view(world, bmax, rows.shape[1])
    return torch.cat([out[r, : e - s] for r, (s, e) in enumerate(sizes)]).to(dev)


def max_over_ranks(value: float, device) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device="cpu" if _gloo() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def finish() -> None:
    """Leave the process group (every rank, before any rank-local tail work such as the CPU baseline)."""
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def barrier(device=None):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and device.type == "cuda" and not _gloo():
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


class GradBuckets:
    """DDP gradient all-reduce of the fine-tune step (config 5; the reference's PL `accelerator: ddp`,
    configs/finetune_ood.yaml:28-30) over ONE flat fp32 gradient buffer.

    The buffer is cut into buckets of ~bucket_bytes, from its END: parameters are laid out in
    declaration (forward) order and the backward produces the last layers' gradients first. Each
    parameter's post-accumulate-grad hook counts down its bucket; a bucket whose gradients are all
    accumulated becomes ready, and ready buckets are all-reduced asynchronously strictly in bucket
    index order (a cursor, as torch DDP does): whatever order the hooks fire in on a rank, every rank
    issues the same sequence of collectives, so RCCL never pairs mismatched buckets. RCCL overlaps them
    with the rest of the backward; finish() launches the remaining buckets (in order), waits, and
    averages. xGMI rings are per-link bound (7 links x ~153 GB/s):
    a few tens of MB per bucket keeps each collective long enough to run near link rate."""

    def __init__(self, grad_flat: torch.Tensor, params, bucket_bytes: int = 32 << 20, group=None):
        """params: [(leaf tensor, offset, numel)] in the buffer's layout order."""
        self.grad, self.group = grad_flat, group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        cap = max(1, bucket_bytes // grad_flat.element_size())
        self.buckets = []          # [lo, hi) element ranges of the flat buffer, launch order
        self.owner = {}
        self.count = []
        cur_hi, cur_lo, members = None, None, 0
        for p, off, n in reversed(list(params)):
            if cur_hi is None:
                cur_hi = off + n
            cur_lo = off
            self.owner[id(p)] = len(self.buckets)
            members += 1
            if cur_hi - cur_lo >= cap:
                self.buckets.append((cur_lo, cur_hi))
                self.count.append(members)
                cur_hi, members = None, 0
        if cur_hi is not None:
            self.buckets.append((cur_lo, cur_hi))
            self.count.append(members)
        # gradients arrive through AccumulateGrad (post-accumulate hook) or, for parameters with a
        # direct gradient view (autograd.direct_grad_view), from the backward kernels' caller
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_hook) for p, _, _ in params]
        self._params = [p for p, _, _ in params]
        for p in self._params:
            p._rdeic_notify = self._on_grad
        self.pending, self.handles, self.fired = [], {}, {}
        self.next_bucket = 0
        self.launch_order = []  # bucket ids in the order their collectives were issued (tests)

    def begin(self):
        self.pending = list(self.count)
        self.handles = {}
        self.fired = {}
        self.next_bucket = 0
        self.launch_order = []

    def _launch(self, b: int):
        if b != self.next_bucket:
            raise RuntimeError(f"bucket {b} launched out of order (next is {self.next_bucket})")
        self.next_bucket += 1
        self.launch_order.append(b)
        lo, hi = self.buckets[b]
        if self.world > 1:
            self.handles[b] = dist.all_reduce(self.grad[lo:hi], group=self.group, async_op=True)
        else:
            self.handles[b] = None

    def _on_hook(self, p):
        if not getattr(p, "_rdeic_direct", False):  # direct-gradient parameters report through _on_grad
            self._on_grad(p)

    def _on_grad(self, p):
        k = id(p)
        self.fired[k] = self.fired.get(k, 0) + 1
        if self.fired[k] > 1:
            raise RuntimeError("a bucketed parameter received two gradient accumulations in one step")
        b = self.owner[k]
        self.pending[b] -= 1
        # launch every consecutive ready bucket from the cursor: a bucket that completes early waits
        # for its predecessors, so the collective sequence is the bucket order on every rank
        while self.next_bucket < len(self.buckets) and self.pending[self.next_bucket] == 0:
            self._launch(self.next_bucket)

    def finish(self):
        while self.next_bucket < len(self.buckets):
            self._launch(self.next_bucket)
        for b in range(len(self.buckets)):
            h = self.handles[b]
            if h is not None:
                h.wait()
        if self.world > 1:
            self.grad.div_(self.world)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for p in self._params:
            if getattr(p, "_rdeic_notify", None) == self._on_grad:
                p._rdeic_notify = None
        self._params = []
