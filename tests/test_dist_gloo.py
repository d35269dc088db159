"""CPU: the N > 1 path (frame sharding + all-gather of padded detections, and the one-collective
per-frame record of detections + counts + embeddings + keypoints) over gloo, exactly
the logic bench.py runs over RCCL, at world sizes 2 and 4 (even and ragged global batches),
and bench.py's own launcher (one child per rank, rendezvous env on 127.0.0.1)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from prpe.dist import shard_range

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


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


def _check(out, world, gb):
    for r in range(world):
        res = torch.load(f"{out}.{r}", weights_only=True)
        gd, gc = res["gd"], res["gc"]
        assert res["rank"] == r and res["world"] == world
        assert gd.shape == (gb, 300, 6) and gc.tolist() == [f % 3 for f in range(gb)]
        for f in range(gb):
            assert torch.all(gd[f, :f % 3] == f) and torch.all(gd[f, f % 3:] == 0)
        rd, rc, ids, emb, kp = res["rec"]
        fr = torch.arange(gb)
        assert torch.equal(rd, gd) and torch.equal(rc, gc) and rc.dtype == torch.int32
        assert ids.dtype == torch.int32 and torch.equal(ids, (fr * 1000003 + 7).to(torch.int32))
        assert emb.shape == (gb, 512) and torch.equal(emb, fr[:, None].float() + torch.arange(512).float()[None] * 1e-3)
        assert kp.shape == (gb, 17, 3) and torch.equal(kp, fr[:, None, None].float() * 0.5 + torch.zeros(gb, 17, 3))


@pytest.mark.parametrize("world,gb", [(2, 6), (4, 7), (4, 3)])
def test_gather_detections_gloo(tmp_path, world, gb):
    port = _free_port()
    out = str(tmp_path / "res")
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_worker.py"), out, str(gb)], env=env))
    for p in procs:
        assert p.wait(timeout=180) == 0
    _check(out, world, gb)


def test_bench_launcher_spawns_ranks(tmp_path, monkeypatch):
    """bench.py --gpus N without WORLD_SIZE: launch_children starts N processes with the
    rendezvous environment (here a gloo worker instead of bench.py itself: no GPU)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    out = str(tmp_path / "res")
    rc = bench.launch_children(3, [sys.executable, os.path.join(HERE, "_dist_worker.py"), out, "5"])
    assert rc == 0
    _check(out, 3, 5)
    for r in range(3):
        assert torch.load(f"{out}.{r}", weights_only=True)["local_rank"] == r
    # a failing rank makes the launcher fail
    assert bench.launch_children(2, [sys.executable, "-c", "import os,sys; sys.exit(int(os.environ['RANK']) + 3)"]) != 0


def test_gathered_parity_gloo(tmp_path):
    """Config 5's rank-0 check (bench.gathered_parity) over gloo, world size 2: CPU stand-in
    ranks make their shard's records with the oracle, the records travel through the same
    all-gathers as in bench.py, rank 0 finds them exact; two frames' records swapped in
    transit are caught (OKS / embedding / NMS mismatch)."""
    port = _free_port()
    out = str(tmp_path / "parity")
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_parity_worker.py"), out, "2", "64"],
                                      env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    res = torch.load(out, weights_only=True)
    good, bad = res["good"], res["bad"]
    assert good["frames"] == [0, 1, 2, 3]
    # same oracle, same frames: equal up to CPU batch-composition rounding (OKS of equal
    # coordinates is 1 - 3e-13 in its float64 arithmetic)
    assert good["oks_delta"] < 1e-9 and good["emb_max_abs"] < 1e-5 and good["cls_max_abs"] < 1e-5
    assert good["nms_exact"] is True
    assert bad["emb_max_abs"] > 1e-3 and bad["nms_exact"] is False and bad["oks_delta"] > 1e-6
