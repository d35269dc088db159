"""GPU: the fused stem + max-pool (prpe_stem_maxpool, csrc/conv_stem.hip; torchvision resnet50
conv1 -> bn1 -> relu -> maxpool, the reference trunk modify_models.py:413-446) against the
unfused path it replaces (prpe_conv2d's chunked stem over the NHWC4 view, then prpe_maxpool):
bit-identical outputs and max|y| slots, partial column strips, flip, run-to-run identity."""
import pytest
import torch

from prpe import engine as E
from prpe import ops, synth
from prpe._lib import PrpeError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(state_dict):
    return E.Engine(state_dict, "cuda")


def _both(eng, x, flip=False):
    with eng.prec("trunk"):
        yf = eng.stem(x, flip, pool=True)
        assert getattr(yf, "_prpe_pooled", False)
        fa = yf._prpe_amax.clone()
        yf = yf.clone()
    E.STEM_POOL = False
    try:
        with eng.prec("trunk"):
            ys = eng.stem(x, flip, pool=True)
            assert not getattr(ys, "_prpe_pooled", False)
            B, H, W, C = ys.shape
            yu = ops.maxpool(ys, torch.empty(B, H // 2, W // 2, C, device="cuda"), 3, 2, 1)
            ua = ys._prpe_amax.clone()
    finally:
        E.STEM_POOL = True
    torch.cuda.synchronize()
    return yf, fa, yu, ua


@pytest.mark.parametrize("N,H,W,flip", [(2, 64, 64, False), (1, 640, 640, False), (3, 96, 136, False),
                                        (2, 640, 640, True)])
def test_stem_maxpool_bit_identical_to_unfused(eng, N, H, W, flip):
    g = torch.Generator().manual_seed(H * 7 + W + N)
    x = torch.rand(N, 3, H, W, generator=g).cuda()
    x[0] *= 3.0                                   # a frame with another range (per-frame scales)
    yf, fa, yu, ua = _both(eng, x, flip)
    assert yf.shape == (N, H // 4, W // 4, 64)
    assert torch.equal(yf, yu), (yf - yu).abs().max().item()
    assert torch.equal(fa, ua)


def test_stem_maxpool_deterministic_and_frame_independent(eng):
    x = synth.frames(48).cuda()
    with eng.prec("trunk"):
        a = eng.stem(x, pool=True).clone()
        b = eng.stem(x, pool=True).clone()
        c = eng.stem(x[[0, 37]].contiguous(), pool=True).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert torch.equal(a[37], c[1]) and torch.equal(a[0], c[0])


def test_stem_maxpool_rejects_bad_shapes(eng):
    with eng.prec("trunk"):
        eng.stem(torch.rand(1, 3, 64, 64).cuda(), pool=True)
    pk = eng._packs["backbone.conv1"]
    buf = torch.zeros(1, 64 + 6, 62 + 8, 4, device="cuda")      # W not a multiple of 4
    with pytest.raises(PrpeError):
        ops.stem_maxpool(buf, 64, 62, torch.ones(1, device="cuda"), pk, torch.empty(1, 16, 15, 64, device="cuda"))
