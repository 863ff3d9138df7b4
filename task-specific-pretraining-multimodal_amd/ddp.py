"""Data parallelism: one process per GPU, gradient all-reduce over RCCL (torch.distributed "nccl").

The reference has no distributed training; this is the build's exchange
step: after the HIP backward has written every gradient into FusedAdam's flat buffer, the buffer is
summed across ranks in fixed-size buckets (reverse parameter order: the head and the last encoder
stages are ready first), and 1/world is folded into Adam's gradient scale, so no separate divide
pass runs.  Per-rank BatchNorm statistics, as PyTorch DDP does by default.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def init_from_env(backend: Optional[str] = None) -> tuple:
    """Initialise the default process group from torchrun-style env vars (RANK, WORLD_SIZE, ...).
    Returns (rank, world_size, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, local


def bucket_views(flat: torch.Tensor, bucket_elems: int) -> List[torch.Tensor]:
    """Split a flat buffer into contiguous buckets, last bucket first (reverse autograd order)."""
    n = flat.numel()
    views = []
    start = 0
    while start < n:
        end = min(n, start + bucket_elems)
        views.append(flat[start:end])
        start = end
    return views[::-1]


class GradAllReduce:
    """Sum the flat gradient buffers of a FusedAdam across ranks (bucketed, in-place)."""

    def __init__(self, flat_grads: List[torch.Tensor], bucket_mb: float = 25.0, group=None):
        self.group = group
        elems = max(1, int(bucket_mb * (1 << 20) / 4))
        self.buckets: List[torch.Tensor] = []
        for f in flat_grads:
            self.buckets += bucket_views(f, elems)

    def __call__(self) -> None:
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        works = [dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group, async_op=True) for b in self.buckets]
        for w in works:
            w.wait()


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every rank start from rank ``src``'s weights and BN buffers."""
    if not dist.is_initialized():
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src=src, group=group)
