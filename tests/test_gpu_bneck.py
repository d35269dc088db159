"""GPU: the fused identity-shortcut bottleneck (prpe_bottleneck, csrc/conv_bneck.hip; ResNet-50
layer1 blocks 1-2, torchvision Bottleneck.forward) against fp64 and against the unfused
precision-3 path (three prpe_conv2d launches with the same packs).

Tolerance: both paths round every conv operand to the precision-3 split (~2^-21); the fused
one rounds t1 / t2 with one scale per 8 x 16 tile instead of per frame, so it is at least as
precise. Bound: max|y - fp64| <= 3x the unfused path's own max error + 2^-22 max|y|."""
import math

import pytest
import torch
import torch.nn.functional as F

from prpe import ops, pack
from prpe._lib import RES_PRE, PrpeError
from test_gpu_ops import DEV, _g, rnd

pytestmark = pytest.mark.gpu


def _packs(seed):
    w1 = rnd(64, 256, 1, 1, seed=seed, scale=1.0 / 16)
    w2 = rnd(64, 64, 3, 3, seed=seed + 1, scale=1.0 / 24)
    w3 = rnd(256, 64, 1, 1, seed=seed + 2, scale=1.0 / 8)
    bn = [(torch.rand(c, generator=_g(seed + 10 + i)) + 0.5, rnd(c, seed=seed + 20 + i, scale=0.3))
          for i, c in enumerate((64, 64, 256))]
    bn[2] = (bn[2][0] * 0.2, bn[2][1])                  # a small last gamma, as the model's
    p1 = pack.pack_conv("c1", w1, 1, 0, DEV, scale=bn[0][0], bias=bn[0][1], act="relu")
    p2 = pack.pack_conv("c2", w2, 1, 1, DEV, scale=bn[1][0], bias=bn[1][1], act="relu")
    p3 = pack.pack_conv("c3", w3, 1, 0, DEV, scale=bn[2][0], bias=bn[2][1], act="relu")
    return (w1, w2, w3), bn, (p1, p2, p3)


def _ref64(x, ws, bn):
    """fp64 torchvision bottleneck on NHWC x (CPU)."""
    t = x.permute(0, 3, 1, 2).double()
    a = t
    for i, (w, (s, b)) in enumerate(zip(ws, bn)):
        a = F.conv2d(a, w.double(), None, 1, 1 if i == 1 else 0) * s.double().view(1, -1, 1, 1) + \
            b.double().view(1, -1, 1, 1)
        a = torch.relu(a) if i < 2 else torch.relu(a + t)
    return a.permute(0, 2, 3, 1)


def _unfused(x, xa, packs):
    N, H, W, _ = x.shape
    t1 = torch.empty(N, H, W, 64, device=DEV)
    t2 = torch.empty(N, H, W, 64, device=DEV)
    y = torch.empty(N, H, W, 256, device=DEV)
    a1, a2 = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
    ops.conv2d(x, packs[0], t1, precision=3, x_amax=xa, y_amax=a1)
    ops.conv2d(t1, packs[1], t2, precision=3, x_amax=a1, y_amax=a2)
    ops.conv2d(t2, packs[2], y, res=x, res_mode=RES_PRE, precision=3, x_amax=a2)
    return y


@pytest.mark.parametrize("N,H,W", [(2, 20, 20), (1, 32, 48), (3, 17, 9), (2, 160, 160)])
def test_bottleneck_fused_vs_fp64_and_unfused(N, H, W):
    ws, bn, packs = _packs(400)
    g = torch.Generator(DEV).manual_seed(N * 1000 + H)
    x = torch.relu(torch.randn(N, H, W, 256, generator=g, device=DEV)) * 2.0
    xa = x.abs().flatten(1).amax(1).contiguous()
    y = torch.empty_like(x)
    ya = torch.zeros(N, device=DEV)
    ops.bottleneck(x, packs, y, xa, ya)
    yu = _unfused(x, xa, packs)
    torch.cuda.synchronize()
    ref = _ref64(x.cpu(), ws, bn)
    e_f = (y.cpu().double() - ref).abs().max().item()
    e_u = (yu.cpu().double() - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"bneck {N}x{H}x{W}: fused {e_f:.2e} unfused {e_u:.2e} max|y| {scale:.2f}")
    assert e_f <= 3 * e_u + 2 ** -22 * scale, (e_f, e_u)
    assert torch.isfinite(y).all()
    # per-frame max|y| slots exactly
    assert torch.equal(ya.cpu(), y.abs().flatten(1).amax(1).cpu())


def test_bottleneck_frames_independent_bit_identical():
    _, _, packs = _packs(410)
    g = torch.Generator(DEV).manual_seed(5)
    x = torch.relu(torch.randn(4, 24, 40, 256, generator=g, device=DEV))
    x[2] *= 50.0                                          # a batch-mate with a very different range
    xa = x.abs().flatten(1).amax(1).contiguous()
    y = torch.empty_like(x)
    ops.bottleneck(x, packs, y, xa)
    y1 = torch.empty_like(x[1:2])
    ops.bottleneck(x[1:2].contiguous(), packs, y1, xa[1:2].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(y[1:2], y1)


def test_bottleneck_rejects_unsupported():
    _, _, packs = _packs(420)
    x = torch.zeros(1, 8, 8, 128, device=DEV)             # wrong width
    with pytest.raises(PrpeError):
        ops.bottleneck(x, packs, torch.empty_like(x), torch.ones(1, device=DEV))


def test_bottleneck_deterministic_large_grid():
    """Run-to-run bit identity at a model-sized grid (96 frames of layer1, 19,200 workgroups, two
    per CU). The compiler once hoisted the next K-step's LDS reads above the barrier that
    publishes the ring stage (conv.h wait_barrier): frames then differed between two bs=256
    forwards in a few thousand of 6.5 M outputs, invisible on small grids."""
    _, _, packs = _packs(430)
    g = torch.Generator(DEV).manual_seed(7)
    x = torch.relu(torch.randn(96, 160, 160, 256, generator=g, device=DEV)) * 2.0
    xa = x.abs().flatten(1).amax(1).contiguous()
    ys = []
    for _ in range(3):
        y = torch.empty_like(x)
        ya = torch.zeros(x.shape[0], device=DEV)
        ops.bottleneck(x, packs, y, xa, ya)
        ys.append((y, ya))
    torch.cuda.synchronize()
    for y, ya in ys[1:]:
        assert torch.equal(y, ys[0][0]) and torch.equal(ya, ys[0][1])


# ---------------------------------------------------------------- projection block (layer1.0)
def _packs_proj(seed):
    w1 = rnd(64, 64, 1, 1, seed=seed, scale=1.0 / 8)
    w2 = rnd(64, 64, 3, 3, seed=seed + 1, scale=1.0 / 24)
    w3 = rnd(256, 64, 1, 1, seed=seed + 2, scale=1.0 / 8)
    wd = rnd(256, 64, 1, 1, seed=seed + 3, scale=1.0 / 8)
    bn = [(torch.rand(c, generator=_g(seed + 10 + i)) + 0.5, rnd(c, seed=seed + 20 + i, scale=0.3))
          for i, c in enumerate((64, 64, 256, 256))]
    p1 = pack.pack_conv("c1", w1, 1, 0, DEV, scale=bn[0][0], bias=bn[0][1], act="relu")
    p2 = pack.pack_conv("c2", w2, 1, 1, DEV, scale=bn[1][0], bias=bn[1][1], act="relu")
    # the engine's pk_dual: W' = [s3 W3 | sd Wd], bias b3 + bd
    wdual = torch.cat([w3.flatten(1) * bn[2][0][:, None], wd.flatten(1) * bn[3][0][:, None]], 1)
    p3 = pack.pack_matrix("c3+ds", wdual, 1, 1, 128, 1, 0, DEV, bias=bn[2][1] + bn[3][1], act="relu")
    return (w1, w2, w3, wd), bn, (p1, p2, p3)


def _ref64_proj(x, ws, bn):
    t = x.permute(0, 3, 1, 2).double()
    aff = lambda a, i: a * bn[i][0].double().view(1, -1, 1, 1) + bn[i][1].double().view(1, -1, 1, 1)
    a = torch.relu(aff(F.conv2d(t, ws[0].double()), 0))
    a = torch.relu(aff(F.conv2d(a, ws[1].double(), None, 1, 1), 1))
    y = torch.relu(aff(F.conv2d(a, ws[2].double()), 2) + aff(F.conv2d(t, ws[3].double()), 3))
    return y.permute(0, 2, 3, 1)


def _unfused_proj(x, xa, packs):
    N, H, W, _ = x.shape
    t1 = torch.empty(N, H, W, 64, device=DEV)
    t2 = torch.empty(N, H, W, 64, device=DEV)
    y = torch.empty(N, H, W, 256, device=DEV)
    a1, a2 = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
    ops.conv2d(x, packs[0], t1, precision=3, x_amax=xa, y_amax=a1)
    ops.conv2d(t1, packs[1], t2, precision=3, x_amax=a1, y_amax=a2)
    ops.conv2d(t2, packs[2], y, precision=3, x_amax=a2, x2=x, x2_amax=xa)
    return y


@pytest.mark.parametrize("N,H,W", [(2, 20, 20), (1, 32, 48), (3, 17, 9), (2, 160, 160)])
def test_bottleneck_proj_fused_vs_fp64_and_unfused(N, H, W):
    ws, bn, packs = _packs_proj(500)
    g = torch.Generator(DEV).manual_seed(N * 1000 + H + 1)
    x = torch.relu(torch.randn(N, H, W, 64, generator=g, device=DEV)) * 2.0
    xa = x.abs().flatten(1).amax(1).contiguous()
    y = torch.empty(N, H, W, 256, device=DEV)
    ya = torch.zeros(N, device=DEV)
    ops.bottleneck(x, packs, y, xa, ya)
    yu = _unfused_proj(x, xa, packs)
    torch.cuda.synchronize()
    ref = _ref64_proj(x.cpu(), ws, bn)
    e_f = (y.cpu().double() - ref).abs().max().item()
    e_u = (yu.cpu().double() - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"bneck proj {N}x{H}x{W}: fused {e_f:.2e} unfused {e_u:.2e} max|y| {scale:.2f}")
    assert e_f <= 3 * e_u + 2 ** -22 * scale, (e_f, e_u)
    assert torch.isfinite(y).all()
    assert torch.equal(ya.cpu(), y.abs().flatten(1).amax(1).cpu())


def test_bottleneck_proj_frames_independent_and_deterministic():
    _, _, packs = _packs_proj(510)
    g = torch.Generator(DEV).manual_seed(9)
    x = torch.relu(torch.randn(96, 160, 160, 64, generator=g, device=DEV))
    x[2] *= 50.0                                          # a batch-mate with a very different range
    xa = x.abs().flatten(1).amax(1).contiguous()
    ys = []
    for _ in range(2):
        y = torch.empty(96, 160, 160, 256, device=DEV)
        ops.bottleneck(x, packs, y, xa)
        ys.append(y)
    y1 = torch.empty(1, 160, 160, 256, device=DEV)
    ops.bottleneck(x[1:2].contiguous(), packs, y1, xa[1:2].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1])
    assert torch.equal(ys[0][1:2], y1)


def test_bottleneck_proj_rejects_wrong_dual_pack():
    _, _, packs = _packs_proj(520)
    _, _, ident = _packs(521)
    x = torch.zeros(1, 8, 8, 64, device=DEV)
    with pytest.raises(PrpeError):                        # conv3 pack without the projection half
        ops.bottleneck(x, (packs[0], packs[1], ident[2]), torch.empty(1, 8, 8, 256, device=DEV),
                       torch.ones(1, device=DEV))


# ---------------------------------------------------------------- layer2 identity blocks (mid 128)
def _packs128(seed):
    w1 = rnd(128, 512, 1, 1, seed=seed, scale=1.0 / 22)
    w2 = rnd(128, 128, 3, 3, seed=seed + 1, scale=1.0 / 34)
    w3 = rnd(512, 128, 1, 1, seed=seed + 2, scale=1.0 / 11)
    bn = [(torch.rand(c, generator=_g(seed + 10 + i)) + 0.5, rnd(c, seed=seed + 20 + i, scale=0.3))
          for i, c in enumerate((128, 128, 512))]
    bn[2] = (bn[2][0] * 0.2, bn[2][1])
    p1 = pack.pack_conv("c1", w1, 1, 0, DEV, scale=bn[0][0], bias=bn[0][1], act="relu")
    p2 = pack.pack_conv("c2", w2, 1, 1, DEV, scale=bn[1][0], bias=bn[1][1], act="relu")
    p3 = pack.pack_conv("c3", w3, 1, 0, DEV, scale=bn[2][0], bias=bn[2][1], act="relu")
    return (w1, w2, w3), bn, (p1, p2, p3)


def _unfused128(x, xa, packs):
    N, H, W, _ = x.shape
    t1 = torch.empty(N, H, W, 128, device=DEV)
    t2 = torch.empty(N, H, W, 128, device=DEV)
    y = torch.empty(N, H, W, 512, device=DEV)
    a1, a2 = torch.zeros(N, device=DEV), torch.zeros(N, device=DEV)
    ops.conv2d(x, packs[0], t1, precision=3, x_amax=xa, y_amax=a1)
    ops.conv2d(t1, packs[1], t2, precision=3, x_amax=a1, y_amax=a2)
    ops.conv2d(t2, packs[2], y, res=x, res_mode=RES_PRE, precision=3, x_amax=a2)
    return y


@pytest.mark.parametrize("N,H,W", [(2, 20, 20), (1, 24, 40), (3, 17, 9), (2, 80, 80)])
def test_bottleneck128_fused_vs_fp64_and_unfused(N, H, W):
    ws, bn, packs = _packs128(600)
    g = torch.Generator(DEV).manual_seed(N * 1000 + H + 2)
    x = torch.relu(torch.randn(N, H, W, 512, generator=g, device=DEV)) * 2.0
    xa = x.abs().flatten(1).amax(1).contiguous()
    y = torch.empty_like(x)
    ya = torch.zeros(N, device=DEV)
    ops.bottleneck(x, packs, y, xa, ya)
    yu = _unfused128(x, xa, packs)
    torch.cuda.synchronize()
    ref = _ref64(x.cpu(), ws, bn)
    e_f = (y.cpu().double() - ref).abs().max().item()
    e_u = (yu.cpu().double() - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"bneck128 {N}x{H}x{W}: fused {e_f:.2e} unfused {e_u:.2e} max|y| {scale:.2f}")
    assert e_f <= 3 * e_u + 2 ** -22 * scale, (e_f, e_u)
    assert torch.isfinite(y).all()
    assert torch.equal(ya.cpu(), y.abs().flatten(1).amax(1).cpu())


def test_bottleneck128_frames_independent_and_deterministic():
    _, _, packs = _packs128(610)
    g = torch.Generator(DEV).manual_seed(11)
    x = torch.relu(torch.randn(96, 80, 80, 512, generator=g, device=DEV))
    x[2] *= 50.0
    xa = x.abs().flatten(1).amax(1).contiguous()
    ys = []
    for _ in range(2):
        y = torch.empty_like(x)
        ops.bottleneck(x, packs, y, xa)
        ys.append(y)
    y1 = torch.empty_like(x[1:2])
    ops.bottleneck(x[1:2].contiguous(), packs, y1, xa[1:2].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1])
    assert torch.equal(ys[0][1:2], y1)
