"""CPU: host logic of the eval-step mirrors (no device calls)."""
import torch

from oracle import model_ref as R
from prpe.evalsteps import COCO_FLIP_PAIRS, flip_partner


def test_flip_partner_is_an_involution():
    p = flip_partner(17)
    assert p[0] == -1
    for a, b in COCO_FLIP_PAIRS:
        assert p[a] == b and p[b] == a


def test_reference_flip_pairs_reverse_the_batch():
    """module.py:482-483 ``flipped[:, pair] = flipped[:, pair].flip(0)``: for paired channels
    the batch order is reversed (not the pair's channels swapped) -- the device kernel's
    mode 0 reproduces exactly this index map."""
    B, K, H, W = 3, 17, 2, 5
    h = torch.zeros(B, K, H, W)
    f = torch.arange(B * K * H * W, dtype=torch.float32).view(B, K, H, W)
    out = R.pose_flip_average(h, f.clone(), "reference") * 2
    part = flip_partner(K)
    for b in range(B):
        for k in range(K):
            b2 = B - 1 - b if part[k] >= 0 else b
            assert torch.equal(out[b, k], torch.flip(f[b2, k], dims=[-1]))
    swap = R.pose_flip_average(h, f.clone(), "swap") * 2
    for k in range(K):
        k2 = part[k] if part[k] >= 0 else k
        assert torch.equal(swap[:, k], torch.flip(f[:, k2], dims=[-1]))
