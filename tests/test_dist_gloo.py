"""CPU: the N > 1 path (frame sharding + all-gather of padded detections) with world_size 2
over gloo, exactly the logic bench.py runs over RCCL."""
import os
import socket
import subprocess
import sys

import torch

from prpe.dist import shard_range

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_covers_batch_exactly():
    for gb in (1, 7, 256, 2048):
        for w in (1, 2, 3, 8):
            r = [shard_range(gb, w, k) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == gb
            assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
            assert max(e - s for s, e in r) - min(e - s for s, e in r) <= 1


def test_gather_detections_world2_gloo(tmp_path):
    port = _free_port()
    out = str(tmp_path / "res")
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_worker.py"), out], env=env))
    for p in procs:
        assert p.wait(timeout=180) == 0
    for r in range(2):
        res = torch.load(f"{out}.{r}", weights_only=True)
        gd, gc = res["gd"], res["gc"]
        assert gd.shape == (6, 300, 6) and gc.tolist() == [f % 3 for f in range(6)]
        for f in range(6):
            assert torch.all(gd[f, :f % 3] == f) and torch.all(gd[f, f % 3:] == 0)
