"""Multi-GPU frame sharding + the one exchange of the path.

Frames are independent in eval mode (BN uses running statistics; the YOLO normalisation is
per sample, modify_models.py:84-85; the precision-3 activation scales are per frame,
engine.Engine.amax_slot), so a global batch shards contiguously over ranks with no
collective on the data path. The exchange is the all-gather of each rank's padded
detections [B_local, max_det, 6] + counts [B_local] (RCCL over xGMI with backend "nccl" on
ROCm; gloo on CPU for tests), giving every rank the whole batch's detections in frame order.
A ragged global batch (B_global % world != 0) is padded to the largest shard for the
collective and trimmed afterwards.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


def shard_range(global_batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, end) of the global batch owned by ``rank`` (balanced, ragged ok)."""
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_tensor(t: torch.Tensor, global_batch: int | None = None, group=None) -> torch.Tensor:
    """All-gather the per-rank shard ``t`` [b_r, ...] along dim 0 -> [B_global, ...] in rank
    (= frame) order. ``global_batch``: total frames when the shards may be ragged (the shard
    of rank r is shard_range(global_batch, world, r)); None = equal shards."""
    world = dist.get_world_size(group)
    if world == 1:
        return t
    if global_batch is None:
        sizes = [t.shape[0]] * world
    else:
        sizes = [e - s for s, e in (shard_range(global_batch, world, r) for r in range(world))]
        me = dist.get_rank(group)
        if t.shape[0] != sizes[me]:
            raise ValueError(f"rank {me} holds {t.shape[0]} frames, shard_range says {sizes[me]}")
    cap = max(sizes)
    t = t.contiguous()
    if t.shape[0] < cap:                                  # pad the ragged shard
        t = torch.cat([t, t.new_zeros((cap - t.shape[0],) + tuple(t.shape[1:]))], 0)
    if dist.get_backend(group) == "nccl":
        g = torch.empty((world * cap,) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
        dist.all_gather_into_tensor(g, t, group=group)
        parts = list(g.split(cap, 0))
    else:
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
    if all(s == cap for s in sizes):
        return torch.cat(parts, 0)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)], 0)


def gather_detections(dets: torch.Tensor, counts: torch.Tensor, global_batch: int | None = None, group=None):
    """All-gather per-rank (dets [b,D,6], counts [b]) -> ([B_global,D,6], [B_global])."""
    return gather_tensor(dets, global_batch, group), gather_tensor(counts, global_batch, group)


def gather_frame_records(parts, global_batch: int | None = None, group=None):
    """All-gather several per-frame tensors in ONE collective (xGMI is point-to-point: one
    larger all-gather instead of one per tensor). ``parts``: tensors [b, ...] of float32 or
    int32 (bit-cast into the fp32 record, so integers travel exactly); returns the gathered
    tensors [B_global, ...] with their dtypes and shapes. SURVEY.md §8e: detections + counts,
    optionally embeddings [b,512] and keypoints + scores [b,17,3] (~9.5 KB per frame)."""
    if dist.get_world_size(group) == 1:
        return list(parts)
    b = parts[0].shape[0]
    flat = []
    for t in parts:
        if t.shape[0] != b or t.dtype not in (torch.float32, torch.int32):
            raise ValueError("gather_frame_records: [b, ...] float32 / int32 tensors of one batch")
        # explicit per-frame width: an empty shard (global batch < world) has b = 0
        flat.append(t.contiguous().view(torch.float32).reshape(b, math.prod(t.shape[1:])))
    rec = gather_tensor(torch.cat(flat, 1), global_batch, group)
    out, o = [], 0
    for t, f in zip(parts, flat):
        w = f.shape[1]
        out.append(rec[:, o:o + w].contiguous().view(t.dtype).reshape((rec.shape[0],) + tuple(t.shape[1:])))
        o += w
    return out

