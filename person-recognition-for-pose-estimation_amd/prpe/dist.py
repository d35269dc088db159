"""Multi-GPU frame sharding + the one exchange of the path.

Frames are independent in eval mode (BN uses running statistics; the YOLO normalisation is
per sample, modify_models.py:84-85), so a global batch shards contiguously over ranks with
no collective on the data path. The exchange is the all-gather of each rank's padded
detections [B_local, max_det, 6] + counts [B_local] (RCCL over xGMI with backend "nccl" on
ROCm; gloo on CPU for tests), giving every rank the whole batch's detections in frame order.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(global_batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, end) of the global batch owned by ``rank`` (balanced, ragged ok)."""
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_detections(dets: torch.Tensor, counts: torch.Tensor, group=None):
    """All-gather equal-shaped per-rank (dets [b,D,6], counts [b]) -> ([W*b,D,6], [W*b])."""
    world = dist.get_world_size(group)
    if world == 1:
        return dets, counts
    if dist.get_backend(group) == "nccl":
        gd = torch.empty((world * dets.shape[0],) + tuple(dets.shape[1:]), device=dets.device, dtype=dets.dtype)
        gc = torch.empty((world * counts.shape[0],), device=counts.device, dtype=counts.dtype)
        dist.all_gather_into_tensor(gd, dets.contiguous(), group=group)
        dist.all_gather_into_tensor(gc, counts.contiguous(), group=group)
        return gd, gc
    ld = [torch.empty_like(dets) for _ in range(world)]
    lc = [torch.empty_like(counts) for _ in range(world)]
    dist.all_gather(ld, dets.contiguous(), group=group)
    dist.all_gather(lc, counts.contiguous(), group=group)
    return torch.cat(ld, 0), torch.cat(lc, 0)
