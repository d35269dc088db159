"""Worker of tests/test_dist_gloo.py (one process per rank, gloo, 127.0.0.1)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "person-recognition-for-pose-estimation_amd"))
from prpe.dist import gather_detections, shard_range  # noqa: E402


def main():
    rank, world, out = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), sys.argv[1]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = shard_range(6, world, rank)
        dets = torch.zeros(e - s, 300, 6)
        cnt = torch.zeros(e - s, dtype=torch.int32)
        for i, f in enumerate(range(s, e)):   # frame f has (f % 3) boxes valued f
            cnt[i] = f % 3
            dets[i, :f % 3] = float(f)
        gd, gc = gather_detections(dets, cnt)
        torch.save({"gd": gd, "gc": gc}, f"{out}.{rank}")
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
