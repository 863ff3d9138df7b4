"""Data parallelism: one process per GPU, gradient all-reduce over RCCL (torch.distributed "nccl").

The reference has no distributed training; this is the build's exchange
step.  The HIP backward writes every gradient into FusedAdam's flat buffer; the buffer is summed
across ranks in buckets and 1/world is folded into Adam's gradient scale, so no divide pass runs.
Per-rank BatchNorm statistics, as PyTorch DDP does by default.

Overlap with backward (PhasedGradAllReduce): FusedTrainStep splits the backward in two phases —
the head, both encoders' fc, layer4 and layer3 (94 % of the 32.6 M gradients, ready first), then
layer2, layer1 and the stems.  The phase-1 gradient ranges are all-reduced on RCCL's stream while
the phase-2 backward runs on the compute stream; only the small phase-2 remainder is exposed.
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


def flat_ranges(offsets: List[int], numels: List[int], total: int, selected: List[bool]) -> List[tuple]:
    """Maximal contiguous [start, end) element ranges of a flat buffer covering the selected
    parameters (offsets: each parameter's start; a parameter's slot runs to the next offset, the
    last to `total`, so alignment padding travels with it)."""
    out = []
    for i, sel in enumerate(selected):
        if not sel:
            continue
        start = offsets[i]
        end = offsets[i + 1] if i + 1 < len(offsets) else total
        if out and out[-1][1] == start:
            out[-1] = (out[-1][0], end)
        else:
            out.append((start, end))
    return out


class PhasedGradAllReduce:
    """Bucketed in-place sum of gradient ranges across ranks, launched per backward phase so that a
    phase's buckets travel (RCCL stream) while the next phase computes (current stream).

    phases: list (one per backward phase) of lists of flat views.  launch(k) enqueues phase k's
    all-reduces (each waits for the work already on the current stream); wait(works) makes the
    current stream wait for them.  With world size 1 nothing is launched unless force=True."""

    def __init__(self, phases: List[List[torch.Tensor]], bucket_mb: float = 64.0, group=None, force: bool = False):
        self.group = group
        self.force = force
        elems = max(1, int(bucket_mb * (1 << 20) / 4))
        self.phases: List[List[torch.Tensor]] = []
        for views in phases:
            bs: List[torch.Tensor] = []
            for v in views:
                bs += bucket_views(v, elems)
            self.phases.append(bs)

    def active(self) -> bool:
        return dist.is_initialized() and (self.force or dist.get_world_size(self.group) > 1)

    def launch(self, k: int) -> list:
        if not self.active():
            return []
        return [dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group, async_op=True) for b in self.phases[k]]

    @staticmethod
    def wait(works: list) -> None:
        for w in works:
            w.wait()


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every rank start from rank ``src``'s weights and BN buffers."""
    if not dist.is_initialized():
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src=src, group=group)
