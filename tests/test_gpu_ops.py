"""GPU: every HIP kernel of the hot path against a plain PyTorch fp32 CPU reference of the
same op (floating-point kernels), at the shapes/variants the model uses.

Tolerances (stated per test): the conv/GEMM path computes in split-bf16 x3 MFMA with fp32
accumulation, i.e. each product to ~2^-17 relative; we allow |d| <= 2e-5 * (sum |a*b|)
scale via rtol/atol on O(1) data. Memory-bound kernels are fp32 VALU: ~1e-6.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from prpe import ops, pack
from prpe._lib import RES_POST, RES_PRE, PrpeError

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _g(seed):
    g = torch.Generator().manual_seed(seed)
    return g


def rnd(*shape, seed=0, scale=1.0):
    return (torch.rand(*shape, generator=_g(seed)) * 2 - 1) * scale


def act_ref(v, act, slope=None):
    if act == "relu":
        return F.relu(v)
    if act == "silu":
        return F.silu(v)
    if act == "gelu":
        return F.gelu(v)
    if act == "prelu":
        return F.prelu(v, slope)
    if act == "sigmoid":
        return torch.sigmoid(v)
    return v


def run_conv(x_nchw, w, stride, pad, act="none", scale=None, bias=None, slope=None, in_s=None, in_b=None,
             res=None, res_mode=0, precision=0, tile=0, x_layout="nhwc", k_order="auto"):
    co = w.shape[0]
    p = pack.pack_conv("t", w, stride, pad, DEV, scale=scale, bias=bias, slope=slope, in_scale=in_s,
                       in_bias=in_b, act=act, k_order=k_order)
    if x_layout == "nchw":
        xd = ops.nhwc(x_nchw.to(DEV))
    else:
        xd = x_nchw.permute(0, 2, 3, 1).contiguous().to(DEV)
    B, _, H, W = x_nchw.shape
    Ho = (H + 2 * pad - w.shape[2]) // stride + 1
    Wo = (W + 2 * pad - w.shape[3]) // stride + 1
    y = torch.empty(B, Ho, Wo, co, device=DEV)
    r = res.permute(0, 2, 3, 1).contiguous().to(DEV) if res is not None else None
    ops.conv2d(xd, p, y, res=r, res_mode=res_mode, precision=precision, tile=tile)
    torch.cuda.synchronize()
    return y.permute(0, 3, 1, 2).cpu()


def ref_conv(x, w, stride, pad, act="none", scale=None, bias=None, slope=None, in_s=None, in_b=None, res=None,
             res_mode=0):
    xx = x.double()
    if in_s is not None:
        xx = xx * in_s.double().view(1, -1, 1, 1) + in_b.double().view(1, -1, 1, 1)
    v = F.conv2d(xx, w.double(), None, stride, pad)
    if scale is not None:
        v = v * scale.double().view(1, -1, 1, 1)
    if bias is not None:
        v = v + bias.double().view(1, -1, 1, 1)
    if res_mode == RES_PRE:
        v = v + res.double()
    v = act_ref(v.float(), act, slope).double()
    if res_mode == RES_POST:
        v = v + res.double()
    return v.float()


def _tol(x, w):
    # bound ~ 2^-16 * sum|x||w| per output; O(1) data -> use a scale-aware atol
    k = w[0].numel()
    return 4e-5 * math.sqrt(k) + 1e-6


@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", [
    (2, 64, 20, 20, 256, 1, 1, 0),      # 1x1
    (2, 64, 17, 19, 96, 3, 1, 1),       # 3x3 ragged spatial, ragged Co
    (2, 32, 20, 20, 64, 3, 2, 1),       # 3x3 / 2
    (1, 256, 10, 10, 512, 1, 2, 0),     # 1x1 / 2 (downsample)
    (2, 8, 40, 40, 16, 3, 1, 1),        # Ci = 8 (YOLO Residual)
    (2, 48, 12, 12, 64, 1, 1, 0),       # Ci = 48 (CSP conv2)
    (1, 512, 7, 7, 64, 7, 1, 0),        # IR-50 output linear as 7x7 conv
])
def test_conv_vector_path(B, Ci, H, W, Co, k, s, p):
    x = rnd(B, Ci, H, W, seed=1)
    w = rnd(Co, Ci, k, k, seed=2, scale=1.0 / math.sqrt(Ci * k * k))
    got = run_conv(x, w, s, p)
    ref = ref_conv(x, w, s, p)
    torch.testing.assert_close(got, ref, rtol=0, atol=_tol(x, w))


@pytest.mark.parametrize("B,H,W,Co,k,s,p", [
    (2, 64, 64, 64, 7, 2, 3),           # ResNet stem (NCHW input, Ci = 3)
    (2, 40, 40, 16, 3, 2, 1),           # YOLO p1
    (2, 64, 48, 768, 16, 16, 2),        # ViT patch embed (k16 s16 pad 2)
])
def test_conv_scalar_path_nchw_input(B, H, W, Co, k, s, p):
    x = rnd(B, 3, H, W, seed=3)
    w = rnd(Co, 3, k, k, seed=4, scale=1.0 / math.sqrt(3 * k * k))
    got = run_conv(x, w, s, p, x_layout="nchw")
    ref = ref_conv(x, w, s, p)
    torch.testing.assert_close(got, ref, rtol=0, atol=_tol(x, w))


@pytest.mark.parametrize("act", ["relu", "silu", "gelu", "prelu", "sigmoid"])
def test_conv_epilogue_acts_and_affine(act):
    Ci, Co = 32, 40
    x = rnd(2, Ci, 9, 11, seed=5)
    w = rnd(Co, Ci, 3, 3, seed=6, scale=0.1)
    sc = torch.rand(Co, generator=_g(7)) + 0.5
    bi = rnd(Co, seed=8)
    sl = torch.rand(Co, generator=_g(9)) * 0.4
    got = run_conv(x, w, 1, 1, act=act, scale=sc, bias=bi, slope=sl if act == "prelu" else None)
    ref = ref_conv(x, w, 1, 1, act=act, scale=sc, bias=bi, slope=sl)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-4)


@pytest.mark.parametrize("mode", [RES_PRE, RES_POST])
def test_conv_residual_modes(mode):
    x = rnd(2, 64, 10, 10, seed=10)
    w = rnd(64, 64, 3, 3, seed=11, scale=0.05)
    r = rnd(2, 64, 10, 10, seed=12)
    got = run_conv(x, w, 1, 1, act="relu", res=r, res_mode=mode)
    ref = ref_conv(x, w, 1, 1, act="relu", res=r, res_mode=mode)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-4)


def test_conv_prologue_affine_zero_padding():
    """IR-50 pre-BN: affine applied to in-bounds taps only; padding stays 0 (net_adaface.py:159)."""
    x = rnd(2, 64, 8, 8, seed=13)
    w = rnd(32, 64, 3, 3, seed=14, scale=0.05)
    s = torch.rand(64, generator=_g(15)) + 0.5
    b = rnd(64, seed=16)
    got = run_conv(x, w, 1, 1, in_s=s, in_b=b)
    ref = ref_conv(x, w, 1, 1, in_s=s, in_b=b)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-4)


@pytest.mark.parametrize("k_order", [0, 1])
@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6])
def test_conv_every_tile_config(tile, k_order):
    x = rnd(2, 64, 9, 13, seed=17)
    w = rnd(150, 64, 3, 3, seed=18, scale=0.05)
    got = run_conv(x, w, 1, 1, tile=tile, k_order=k_order)
    ref = ref_conv(x, w, 1, 1)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-4)


@pytest.mark.parametrize("precision", [0, 1, 2])
@pytest.mark.parametrize("tile", [5, 6])
def test_conv_256_row_tiles_chunked_epilogue(tile, precision):
    """256-row tiles stage the C tile through LDS in row chunks (fewer rows fit when the ring
    holds fewer planes); residual + PReLU exercise the vector epilogue across chunk borders."""
    x = rnd(3, 96, 13, 17, seed=60)
    w = rnd(136, 96, 3, 3, seed=61, scale=0.03)
    r = rnd(3, 136, 13, 17, seed=62)
    sc = torch.rand(136, generator=_g(63)) + 0.5
    bi = rnd(136, seed=64)
    sl = torch.rand(136, generator=_g(65)) * 0.4
    got = run_conv(x, w, 1, 1, act="prelu", scale=sc, bias=bi, slope=sl, res=r, res_mode=RES_PRE,
                   precision=precision, tile=tile)
    ref = ref_conv(x, w, 1, 1, act="prelu", scale=sc, bias=bi, slope=sl, res=r, res_mode=RES_PRE)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-2 if precision == 1 else 2e-4)


@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", [
    (2, 64, 17, 19, 96, 3, 1, 1),
    (2, 128, 11, 9, 64, 3, 2, 1),
    (1, 512, 7, 7, 64, 7, 1, 0),
    (2, 32, 10, 10, 40, 5, 1, 2),
])
def test_conv_chunk_major_matches_tap_major(B, Ci, H, W, Co, k, s, p):
    """k_order 1 (chunk-major K) is a pure re-ordering of the reduction: same result as
    tap-major within rounding, for 3x3/5x5/7x7 and strided convs, with the IR-50 prologue."""
    x = rnd(B, Ci, H, W, seed=66)
    w = rnd(Co, Ci, k, k, seed=67, scale=1.0 / math.sqrt(Ci * k * k))
    s_in = torch.rand(Ci, generator=_g(68)) + 0.5
    b_in = rnd(Ci, seed=69)
    ref = ref_conv(x, w, s, p, in_s=s_in, in_b=b_in)
    for ko in (0, 1):
        got = run_conv(x, w, s, p, in_s=s_in, in_b=b_in, k_order=ko, precision=2)
        torch.testing.assert_close(got, ref, rtol=0, atol=1e-5)


def test_conv_chunk_major_rejects_unaligned_input():
    """k_order 1 needs channel-contiguous 16-B aligned rows: a channel-offset view fails loudly."""
    big = rnd(1, 6, 6, 66, seed=70).to(DEV)
    xin = big[..., 2:66]                        # 64 channels at an 8-B offset
    w = rnd(8, 64, 3, 3, seed=71)
    p = pack.pack_conv("t", w, 1, 1, DEV, k_order=1)
    with pytest.raises(PrpeError):
        ops.conv2d(xin, p, torch.empty(1, 6, 6, 8, device=DEV))


def test_conv_strided_views_in_and_out():
    """Input = channel slice of a concat buffer, output written into another slice."""
    big = rnd(2, 10, 10, 96, seed=19).to(DEV)
    xin = big[..., 32:96]                      # 64 channels, channel stride 1, pixel stride 96
    w = rnd(24, 64, 3, 3, seed=20, scale=0.05)
    p = pack.pack_conv("t", w, 1, 1, DEV)
    out = torch.zeros(2, 10, 10, 80, device=DEV)
    ops.conv2d(xin, p, out[..., 40:64])
    torch.cuda.synchronize()
    ref = ref_conv(xin.cpu().permute(0, 3, 1, 2), w, 1, 1)
    torch.testing.assert_close(out[..., 40:64].cpu().permute(0, 3, 1, 2), ref, rtol=0, atol=2e-4)
    assert torch.all(out[..., :40] == 0) and torch.all(out[..., 64:] == 0)


def test_conv_precision_modes_ordering():
    """plain bf16 >> 2-plane split (~2^-17) >> 3-plane split (fp32-faithful, ~fp32 rounding)."""
    x = rnd(1, 256, 16, 16, seed=21)
    w = rnd(128, 256, 3, 3, seed=22, scale=0.02)
    ref = ref_conv(x, w, 1, 1)                      # fp64 accumulate
    e3 = (run_conv(x, w, 1, 1, precision=0) - ref).abs().max().item()
    e1 = (run_conv(x, w, 1, 1, precision=1) - ref).abs().max().item()
    e6 = (run_conv(x, w, 1, 1, precision=2) - ref).abs().max().item()
    f32 = (F.conv2d(x, w, None, 1, 1) - ref).abs().max().item()   # CPU fp32 itself
    assert e3 < e1 / 50, (e3, e1)
    assert e6 < e3, (e6, e3)
    # fp32 accumulation of K = 2304 terms in one MFMA accumulator: ~sqrt(K)*2^-24*|y|
    # (mkldnn's blocked fp32 sums are ~6x tighter on this shape)
    assert e6 <= 10 * f32 + 1e-6, (e6, f32)


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6])
def test_conv_fp32_faithful_mode_every_tile(tile):
    x = rnd(2, 64, 9, 13, seed=46)
    w = rnd(150, 64, 3, 3, seed=47, scale=0.05)
    got = run_conv(x, w, 1, 1, precision=2, tile=tile, act="relu")
    ref = ref_conv(x, w, 1, 1, act="relu")
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-6)


WAVE_SHAPES = [
    (2, 64, 17, 19, 96, 3, 1, 1),       # ragged spatial (M tail inside a wave), ragged Co
    (2, 128, 11, 9, 64, 3, 2, 1),       # 3x3 / 2
    (2, 64, 20, 20, 256, 1, 1, 0),      # 1x1, two column tiles
    (1, 256, 10, 10, 512, 1, 2, 0),     # 1x1 / 2 (downsample)
    (1, 512, 7, 7, 64, 7, 1, 0),        # 7x7 (IR-50 output linear)
    (3, 96, 13, 17, 136, 3, 1, 1),      # Co beyond one 128 tile
]


@pytest.mark.parametrize("precision", [0, 2])
@pytest.mark.parametrize("tile", [21, 22, 23, 24, 25, 26])
@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", WAVE_SHAPES)
def test_conv_wave_kernel_bit_exact_vs_lds_staged(B, Ci, H, W, Co, k, s, p, tile, precision):
    """conv_wave.hip (A straight into fragment registers, B through an LDS-DMA ring) runs the
    same K order, plane split and MFMA order per accumulator as the register-staged kernel:
    the results agree bit for bit, and both match the fp64 reference."""
    x = rnd(B, Ci, H, W, seed=80)
    w = rnd(Co, Ci, k, k, seed=81, scale=1.0 / math.sqrt(Ci * k * k))
    sc = torch.rand(Co, generator=_g(82)) + 0.5
    bi = rnd(Co, seed=83)
    kw = dict(act="silu", scale=sc, bias=bi, k_order=1, precision=precision)
    got = run_conv(x, w, s, p, tile=tile, **kw)
    base = run_conv(x, w, s, p, tile=5, **kw)
    assert torch.equal(got, base)
    ref = ref_conv(x, w, s, p, act="silu", scale=sc, bias=bi)
    torch.testing.assert_close(got, ref, rtol=0, atol=_tol(x, w) * 2)


@pytest.mark.parametrize("precision,tile", [(3, 23), (3, 25), (3, 26), (3, 27), (0, 23), (0, 28)])
@pytest.mark.parametrize("B,H,W,Ci,Co", [(2, 17, 19, 64, 96), (3, 11, 13, 256, 256), (1, 40, 40, 128, 512)])
def test_conv_wave_pixel_contiguous_1x1_bit_exact(B, H, W, Ci, Co, precision, tile):
    """1x1 / stride-1 convs over a dense input take conv_wave's pixel-contiguous A path (X11: lane
    quads on 64 contiguous bytes, transposed to the fragment layout through LDS, rows past M
    beyond the descriptor); the same conv over a cropped view of a larger buffer (not dense)
    takes the fragment-lane loads. Bit-identical (ragged M tails and a pre-activation residual
    included), and both at the fp64 reference's tolerance."""
    x = (torch.rand(B, H, W, Ci, generator=_g(90)) * 2 - 1).to(DEV)
    big = torch.zeros(B, H + 2, W + 3, Ci, device=DEV)
    big[:, 1:H + 1, 2:W + 2] = x
    xv = big[:, 1:H + 1, 2:W + 2]
    w = rnd(Co, Ci, 1, 1, seed=91, scale=1.0 / math.sqrt(Ci))
    sc = torch.rand(Co, generator=_g(92)) + 0.5
    bi = rnd(Co, seed=93)
    pk = pack.pack_conv("t", w, 1, 0, DEV, scale=sc, bias=bi, act="relu")
    r = (torch.rand(B, H, W, Co, generator=_g(94)) - 0.5).to(DEV)
    xa = x.abs().flatten(1).amax(1).contiguous()
    outs = []
    for xin in (x, xv):
        y = torch.empty(B, H, W, Co, device=DEV)
        ops.conv2d(xin, pk, y, res=r, res_mode=RES_PRE, precision=precision, tile=tile,
                   x_amax=xa if precision == 3 else None)
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = ref_conv(x.permute(0, 3, 1, 2).cpu(), w, 1, 0, act="relu", scale=sc, bias=bi,
                   res=r.permute(0, 3, 1, 2).cpu(), res_mode=RES_PRE)
    torch.testing.assert_close(outs[0].permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=_tol(x, w) * 2)


@pytest.mark.parametrize("precision,tile", [(3, 23), (3, 25), (3, 27), (0, 23), (0, 28)])
@pytest.mark.parametrize("B,H,W,Ci,Co,s", [(2, 17, 19, 64, 96, 1), (3, 12, 10, 128, 256, 1), (2, 20, 20, 256, 256, 2),
                                           (1, 40, 40, 64, 128, 1)])
def test_conv_wave_unpadded_over_zero_border_bit_exact(B, H, W, Ci, Co, s, precision, tile):
    """The trunk's 3x3 conv2 over a zero-bordered copy of its input with pad 0 (engine
    T1_BORDER: no tap masks, conv_wave's pixel-contiguous A loads, XM 2) equals the pad-1 conv
    over the plain input (fragment-lane loads with tap masks) bit for bit, stride 2 included."""
    x = (torch.rand(B, H, W, Ci, generator=_g(95)) * 2 - 1).to(DEV)
    xb = torch.zeros(B, H + 2, W + 2, Ci, device=DEV)
    xb[:, 1:H + 1, 1:W + 1] = x
    w = rnd(Co, Ci, 3, 3, seed=96, scale=1.0 / math.sqrt(Ci * 9))
    sc = torch.rand(Co, generator=_g(97)) + 0.5
    bi = rnd(Co, seed=98)
    xa = x.abs().flatten(1).amax(1).contiguous()
    outs = []
    for xin, pad in ((x, 1), (xb, 0)):
        pk = pack.pack_conv("t", w, s, pad, DEV, scale=sc, bias=bi, act="relu", k_order=1)
        Ho, Wo = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
        y = torch.empty(B, Ho, Wo, Co, device=DEV)
        ops.conv2d(xin, pk, y, precision=precision, tile=tile, x_amax=xa if precision == 3 else None)
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = ref_conv(x.permute(0, 3, 1, 2).cpu(), w, s, 1, act="relu", scale=sc, bias=bi)
    torch.testing.assert_close(outs[1].permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=_tol(x, w) * 2)


@pytest.mark.parametrize("precision,tile", [(0, 28), (0, 29), (2, 27)])
@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", WAVE_SHAPES)
def test_conv_wave_two_stage_ring_bit_exact(B, Ci, H, W, Co, k, s, p, tile, precision):
    """The 2-stage B-ring tiles (the automatic wide choice for precision 0 / 2): same K order, plane split and MFMA order per accumulator as the register-staged
    kernel, so bit-identical to it; pre-activation residual included."""
    x = rnd(B, Ci, H, W, seed=80)
    w = rnd(Co, Ci, k, k, seed=81, scale=1.0 / math.sqrt(Ci * k * k))
    sc = torch.rand(Co, generator=_g(82)) + 0.5
    bi = rnd(Co, seed=83)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    # (a 1x1-pixel residual permuted to NHWC keeps unit W/H strides, which the vector epilogue
    # rightly rejects; that shape runs without one)
    r = rnd(B, Co, Ho, Wo, seed=97) if Ho * Wo > 1 else None
    kw = dict(act="gelu", scale=sc, bias=bi, k_order=1, precision=precision, res=r,
              res_mode=RES_PRE if r is not None else 0)
    got = run_conv(x, w, s, p, tile=tile, **kw)
    assert torch.equal(got, run_conv(x, w, s, p, tile=5, **kw))


@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", WAVE_SHAPES)
def test_conv_f16_two_stage_ring_bit_exact(B, Ci, H, W, Co, k, s, p):
    """precision 3: the 2-stage 128x128 tile (27, the automatic wide choice) agrees bit for bit
    with the 3-stage one (26)."""
    x = torch.relu(rnd(B, Ci, H, W, seed=91)) * 7.0
    w = rnd(Co, Ci, k, k, seed=92, scale=1.0 / math.sqrt(Ci * k * k))
    sc = torch.rand(Co, generator=_g(93)) + 0.5
    bi = rnd(Co, seed=94)
    a, ya = _conv_p3(x, w, s, p, tile=27, scale=sc, bias=bi, act="silu")
    b, yb = _conv_p3(x, w, s, p, tile=26, scale=sc, bias=bi, act="silu")
    assert torch.equal(a, b) and ya == yb


HALO_SHAPES = [
    (2, 64, 17, 19, 96, 3, 1, 1),       # ragged in both spatial dims (partial tiles), Co < 128
    (3, 96, 13, 17, 136, 3, 1, 1),      # Co beyond one 128 tile, odd chunk count
    (1, 256, 33, 40, 128, 3, 1, 1),     # 8 chunks (halo double buffer wraps 4 times)
    (2, 32, 16, 16, 256, 3, 1, 1),      # one chunk (no halo prefetch), two Co tiles, exact tiles
]


@pytest.mark.parametrize("tile", [30, 31, 32, 33, 34, 35, 36, 37])
@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", HALO_SHAPES)
def test_conv_halo_kernel_bit_exact_vs_wave(B, Ci, H, W, Co, k, s, p, tile):
    """conv_halo.hip (input patch + halo staged once per 32-channel chunk, A fragments of every
    tap from LDS) runs the wave kernel's K order, split and MFMA order: bit-identical to it,
    with a pre-activation residual and GELU, for fp32 input, planes input and precision 3."""
    x = rnd(B, Ci, H, W, seed=180)
    w = rnd(Co, Ci, k, k, seed=181, scale=1.0 / math.sqrt(Ci * k * k))
    sc = torch.rand(Co, generator=_g(182)) + 0.5
    bi = rnd(Co, seed=183)
    r = rnd(B, Co, H, W, seed=184)
    kw = dict(act="gelu", scale=sc, bias=bi, k_order=1, precision=0, res=r, res_mode=RES_PRE)
    got = run_conv(x, w, s, p, tile=tile, **kw)
    assert torch.equal(got, run_conv(x, w, s, p, tile=28, **kw))
    ref = ref_conv(x, w, s, p, act="gelu", scale=sc, bias=bi, res=r, res_mode=RES_PRE)
    torch.testing.assert_close(got, ref, rtol=0, atol=_tol(x, w) * 2)
    # planes input (the adapters' upconv output format) and planes output
    pk = pack.pack_conv("h", w, 1, 1, DEV, scale=sc, bias=bi, act="gelu", k_order=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    xpl = torch.empty_like(xd)
    ops.conv2d(xd, pack.pack_conv("i", torch.eye(Ci).view(Ci, Ci, 1, 1), 1, 0, DEV), xpl, precision=2,
               y_planes=True)
    outs = []
    for t in (tile, 28):
        y = torch.empty(B, H, W, Co, device=DEV)
        ops.conv2d(xpl, pk, y, precision=0, x_planes=True, tile=t)
        ypl = torch.empty(B, H, W, Co, device=DEV)
        ops.conv2d(xd, pk, ypl, precision=0, y_planes=True, tile=t)
        outs.append((y, ypl))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # precision 3 with per-frame scales and max|y| slots
    xp = torch.relu(x) * 7.0
    a, ya = _conv_p3(xp, w, s, p, tile=tile, scale=sc, bias=bi, act="silu")
    b, yb = _conv_p3(xp, w, s, p, tile=27, scale=sc, bias=bi, act="silu")
    assert torch.equal(a, b) and ya == yb


TAPS_SHAPES = [
    (2, 64, 17, 19, 128, 27),   # ragged tiles, the adapter's n2 = 9 taps x 3 channels
    (1, 256, 24, 20, 96, 12),   # Co < 128 (zero-padded w2 columns), 8 chunks
    (2, 32, 9, 33, 64, 32),     # one chunk, the widest n2
]


@pytest.mark.parametrize("mode", ["fp32", "planes", "p3"])
@pytest.mark.parametrize("B,Ci,H,W,Co,n2", TAPS_SHAPES)
def test_conv_halo_taps_epilogue(B, Ci, H, W, Co, n2, mode):
    """prpe_conv_desc.w2: the haloed-tile kernel's epilogue multiplies its activated tile by
    w2^T on the matrix cores (two bf16 planes per operand, three products: the precision-0
    split) and writes z = y' w2^T to y2 (y untouched). y' is the same conv's unfused output
    (same kernel, bit-identical accumulation), so z is checked against y' w2^T in fp64 within
    the split's bound: each operand carries <= 2^-16 relative residual after two bf16 planes,
    plus fp32 accumulation (2^-24 per term): 2^-14 * sum_k |y'_k w2_ck| covers both."""
    x = rnd(B, Ci, H, W, seed=190)
    if mode == "p3":
        x = torch.relu(x) * 5.0
    w = rnd(Co, Ci, 3, 3, seed=191, scale=1.0 / math.sqrt(Ci * 9))
    sc = torch.rand(Co, generator=_g(192)) + 0.5
    bi = rnd(Co, seed=193)
    w2 = rnd(n2, Co, seed=194).to(DEV)
    pk = pack.pack_conv("t", w, 1, 1, DEV, scale=sc, bias=bi, act="gelu", k_order=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    kw = dict(precision=0)
    if mode == "planes":
        xpl = torch.empty_like(xd)
        ops.conv2d(xd, pack.pack_conv("i", torch.eye(Ci).view(Ci, Ci, 1, 1), 1, 0, DEV), xpl, precision=2,
                   y_planes=True)
        xd, kw = xpl, dict(precision=0, x_planes=True)
    elif mode == "p3":
        kw = dict(precision=3, x_amax=frame_amax(x).to(DEV))
    y = torch.empty(B, H, W, Co, device=DEV)
    ops.conv2d(xd, pk, y, tile=31, **kw)
    sink = torch.full((B, H, W, Co), float("nan"), device=DEV)
    z = torch.full((B, H, W, n2), float("nan"), device=DEV)
    ops.conv2d(xd, pk, sink, w2=w2, y2=z, **kw)
    torch.cuda.synchronize()
    assert torch.isnan(sink).all()
    yd, wd = y.double().cpu(), w2.double().cpu()
    ref = yd @ wd.T
    bound = (yd.abs() @ wd.abs().T) * 2.0 ** -14
    err = (z.double().cpu() - ref).abs()
    assert torch.isfinite(z).all() and bool((err <= bound).all()), float((err / bound.clamp_min(1e-30)).max())
    # only the haloed-tile kernel implements it
    with pytest.raises(PrpeError):
        ops.conv2d(xd, pk, sink, w2=w2, y2=z, tile=28, **kw)


@pytest.mark.parametrize("mode", ["fp32", "planes", "p3"])
@pytest.mark.parametrize("B,Ci,H,W,Co,nmid,n3", [(2, 64, 17, 19, 128, 64, 27), (1, 96, 12, 35, 96, 40, 12)])
def test_conv_halo_taps_two_stage(B, Ci, H, W, Co, nmid, n3, mode):
    """prpe_conv_desc.w3: z1 = act2(scale2 (y' w2^T) + bias2) (w2 [nmid, Co]), then z = z1 w3^T
    (w3 [n3, nmid]) in the haloed-tile kernel's epilogue (the YOLO adapter's .10 -> .13 -> .16
    tap GEMM chain). Checked against fp64 of the same chain on the unfused conv output y', with
    each stage's split-bf16 bound (2^-14 of its sum of |products|) carried through SiLU
    (|silu'| <= 1.1)."""
    x = rnd(B, Ci, H, W, seed=195)
    if mode == "p3":
        x = torch.relu(x) * 5.0
    w = rnd(Co, Ci, 3, 3, seed=196, scale=1.0 / math.sqrt(Ci * 9))
    sc = torch.rand(Co, generator=_g(197)) + 0.5
    bi = rnd(Co, seed=198)
    w2 = rnd(nmid, Co, seed=199, scale=1.0 / math.sqrt(Co)).to(DEV)
    s2 = (torch.rand(nmid, generator=_g(200)) + 0.5).to(DEV)
    b2 = rnd(nmid, seed=201).to(DEV)
    w3 = rnd(n3, nmid, seed=202).to(DEV)
    pk = pack.pack_conv("t", w, 1, 1, DEV, scale=sc, bias=bi, act="silu", k_order=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    kw = dict(precision=0)
    if mode == "planes":
        xpl = torch.empty_like(xd)
        ops.conv2d(xd, pack.pack_conv("i", torch.eye(Ci).view(Ci, Ci, 1, 1), 1, 0, DEV), xpl, precision=2,
                   y_planes=True)
        xd, kw = xpl, dict(precision=0, x_planes=True)
    elif mode == "p3":
        kw = dict(precision=3, x_amax=frame_amax(x).to(DEV))
    y = torch.empty(B, H, W, Co, device=DEV)
    ops.conv2d(xd, pk, y, tile=31, **kw)
    sink = torch.full((B, H, W, Co), float("nan"), device=DEV)
    z = torch.full((B, H, W, n3), float("nan"), device=DEV)
    ops.conv2d(xd, pk, sink, w2=w2, y2=z, w3=w3, scale2=s2, bias2=b2, act2="silu", **kw)
    torch.cuda.synchronize()
    assert torch.isnan(sink).all()
    yd = y.double().cpu()
    w2d, w3d, s2d, b2d = (t.double().cpu() for t in (w2, w3, s2, b2))
    u = (yd @ w2d.T) * s2d + b2d
    z1 = u * torch.sigmoid(u)
    ref = z1 @ w3d.T
    e1 = 1.1 * s2d.abs() * (yd.abs() @ w2d.abs().T) * 2.0 ** -14 + z1.abs() * 2.0 ** -20
    bound = (z1.abs() + e1) @ w3d.abs().T * 2.0 ** -14 + e1 @ w3d.abs().T
    err = (z.double().cpu() - ref).abs()
    assert torch.isfinite(z).all() and bool((err <= bound).all()), float((err / bound.clamp_min(1e-30)).max())
    with pytest.raises(PrpeError):                    # PReLU has no slope vector in the second stage
        ops.conv2d(xd, pk, sink, w2=w2, y2=z, w3=w3, scale2=s2, bias2=b2, act2="prelu", **kw)


@pytest.mark.parametrize("B,Ci,H,Co", [(5, 64, 7, 128), (70, 512, 7, 512), (3, 32, 4, 64), (2, 256, 2, 64)])
def test_conv_splitk_linear(B, Ci, H, Co):
    """conv_splitk.hip (full-window conv = linear over the flattened frame, split along K: the
    IR-50 output layer): prologue BN, epilogue BN + PReLU, ragged frame counts; vs fp64 within
    the precision-0 bound, and the automatic choice (tile 0) takes it for the IR-50 shape."""
    x = rnd(B, Ci, H, H, seed=210)
    w = rnd(Co, Ci, H, H, seed=211, scale=1.0 / math.sqrt(Ci * H * H))
    sc = torch.rand(Co, generator=_g(212)) + 0.5
    bi = rnd(Co, seed=213)
    sl = torch.rand(Co, generator=_g(214)) * 0.3
    ins = torch.rand(Ci, generator=_g(215)) + 0.5
    inb = rnd(Ci, seed=216)
    kw = dict(act="prelu", scale=sc, bias=bi, slope=sl, in_s=ins, in_b=inb, k_order=0)
    got = run_conv(x, w, 1, 0, tile=50, **kw)
    ref = ref_conv(x, w, 1, 0, act="prelu", scale=sc, bias=bi, slope=sl, in_s=ins, in_b=inb)
    xs = x * ins.view(1, -1, 1, 1) + inb.view(1, -1, 1, 1)
    torch.testing.assert_close(got, ref, rtol=0, atol=_tol(xs, w) * 2)
    if Ci * H * H >= 4096:
        assert torch.equal(run_conv(x, w, 1, 0, tile=0, **kw), got)


GEMM_SHAPES = [
    (2, 64, 13, 11, 256),       # M = 286: one full + one ragged 256-row tile, 2 K-steps
    (3, 768, 8, 12, 768),       # ViT-like: K = 768, three column tiles
    (1, 96, 40, 40, 512),       # M = 1600, odd K-step count
    (2, 32, 9, 9, 256),         # one K-step (the pipelined loop's prologue / tail only)
]


@pytest.mark.parametrize("tile", [40, 41, 42, 43, 47, 49])
@pytest.mark.parametrize("B,Ci,H,W,Co", GEMM_SHAPES)
def test_conv_gemm_kernel_bit_exact_vs_wave(B, Ci, H, W, Co, tile):
    """conv_gemm.hip (256 x 256 tile, A and B both LDS-DMA'd) == the wave kernel bit for bit:
    fp32 and planes input, planes output, pre-activation residual, GELU, per-frame max|y|."""
    x = rnd(B, Ci, H, W, seed=190)
    w = rnd(Co, Ci, 1, 1, seed=191, scale=1.0 / math.sqrt(Ci))
    sc = torch.rand(Co, generator=_g(192)) + 0.5
    bi = rnd(Co, seed=193)
    r = rnd(B, Co, H, W, seed=194)
    kw = dict(act="gelu", scale=sc, bias=bi, precision=0, res=r, res_mode=RES_PRE)
    got = run_conv(x, w, 1, 0, tile=tile, **kw)
    assert torch.equal(got, run_conv(x, w, 1, 0, tile=28, **kw))
    ref = ref_conv(x, w, 1, 0, act="gelu", scale=sc, bias=bi, res=r, res_mode=RES_PRE)
    torch.testing.assert_close(got, ref, rtol=0, atol=_tol(x, w) * 2)
    pk = pack.pack_conv("g", w, 1, 0, DEV, scale=sc, bias=bi, act="gelu")
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    xpl = torch.empty_like(xd)
    ops.conv2d(xd, pack.pack_conv("i", torch.eye(Ci).view(Ci, Ci, 1, 1), 1, 0, DEV), xpl, precision=2,
               y_planes=True)
    outs = []
    for t in (tile, 28):
        y = torch.empty(B, H, W, Co, device=DEV)
        ya = torch.zeros(B, device=DEV)
        ops.conv2d(xpl, pk, y, precision=0, x_planes=True, tile=t, y_amax=ya)
        ypl = torch.empty(B, H, W, Co, device=DEV)
        ops.conv2d(xd, pk, ypl, precision=0, y_planes=True, tile=t)
        outs.append((y, ya, ypl))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert torch.equal(outs[0][1].cpu(), frame_amax(outs[0][0]))


def test_conv_gemm_persistent_walks_many_tiles_bit_exact():
    """Tiles 49 / 47 (tiles 40 / 41 persistent: each workgroup walks tiles t, t + G, ... with the next
    tile's first K-steps DMA'd under this tile's epilogue) on a launch with more tiles than workgroups (2 x 399
    x 401 pixels = 1,250 row tiles x 2 column tiles, the last one ragged) == tile 40 bit for bit:
    fp32 and planes input, planes and fp32 output, residual, GELU, per-frame max|y|; and at
    precision 3 (per-row frame scales)."""
    B, Ci, H, W, Co = 2, 64, 399, 401, 256
    x = rnd(B, Ci, H, W, seed=290)
    w = rnd(Co, Ci, 1, 1, seed=291, scale=1.0 / math.sqrt(Ci))
    sc = torch.rand(Co, generator=_g(292)) + 0.5
    bi = rnd(Co, seed=293)
    r = rnd(B, Co, H, W, seed=294)
    kw = dict(act="gelu", scale=sc, bias=bi, precision=0, res=r, res_mode=RES_PRE)
    assert torch.equal(run_conv(x, w, 1, 0, tile=49, **kw), run_conv(x, w, 1, 0, tile=40, **kw))
    assert torch.equal(run_conv(x, w, 1, 0, tile=47, **kw), run_conv(x, w, 1, 0, tile=41, **kw))
    pk = pack.pack_conv("g", w, 1, 0, DEV, scale=sc, bias=bi, act="gelu")
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    xpl = torch.empty_like(xd)
    ops.conv2d(xd, pack.pack_conv("i", torch.eye(Ci).view(Ci, Ci, 1, 1), 1, 0, DEV), xpl, precision=2,
               y_planes=True)
    outs = []
    for t in (49, 40):
        y = torch.empty(B, H, W, Co, device=DEV)
        ya = torch.zeros(B, device=DEV)
        ops.conv2d(xpl, pk, y, precision=0, x_planes=True, tile=t, y_amax=ya)
        ypl = torch.empty(B, H, W, Co, device=DEV)
        ops.conv2d(xd, pk, ypl, precision=0, y_planes=True, tile=t)
        outs.append((y, ya, ypl))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    xr = torch.relu(x) * torch.tensor([7.0, 0.01]).view(B, 1, 1, 1)
    a, ya = _conv_p3(xr, w, 1, 0, tile=49, scale=sc, bias=bi, act="relu", res=r, res_mode=RES_PRE)
    b, yb = _conv_p3(xr, w, 1, 0, tile=40, scale=sc, bias=bi, act="relu", res=r, res_mode=RES_PRE)
    assert torch.equal(a, b) and ya == yb


@pytest.mark.parametrize("B,Ci,H,W,Co", GEMM_SHAPES + [(3, 64, 5, 7, 256)])
def test_conv_gemm_kernel_precision3_bit_exact_vs_wave(B, Ci, H, W, Co):
    """precision 3 on the GEMM kernel (per-row frame scales; the last shape has 35-pixel frames,
    so 256-row tiles straddle up to 8 frames) == the wave kernel's 128x128 tile, with the
    per-frame max|y| slots and a residual."""
    x = torch.relu(rnd(B, Ci, H, W, seed=195)) * torch.tensor([7.0, 0.01, 300.0][:B]).view(B, 1, 1, 1)
    w = rnd(Co, Ci, 1, 1, seed=196, scale=1.0 / math.sqrt(Ci))
    sc = torch.rand(Co, generator=_g(197)) + 0.5
    bi = rnd(Co, seed=198)
    r = rnd(B, Co, H, W, seed=199)
    a, ya = _conv_p3(x, w, 1, 0, tile=40, scale=sc, bias=bi, act="relu", res=r, res_mode=RES_PRE)
    b, yb = _conv_p3(x, w, 1, 0, tile=27, scale=sc, bias=bi, act="relu", res=r, res_mode=RES_PRE)
    assert torch.equal(a, b) and ya == yb


@pytest.mark.parametrize("mode", [RES_PRE, RES_POST])
@pytest.mark.parametrize("tile", [21, 23])
def test_conv_wave_kernel_prologue_residual_prelu(mode, tile):
    """IR-50 pre-BN prologue (padding taps stay 0) + PReLU + residual through the per-wave
    epilogue, including a non-linear residual view (subsampled shortcut)."""
    x = rnd(2, 64, 12, 10, seed=84)
    w = rnd(96, 64, 3, 3, seed=85, scale=0.05)
    s_in = torch.rand(64, generator=_g(86)) + 0.5
    b_in = rnd(64, seed=87)
    sl = torch.rand(96, generator=_g(88)) * 0.4
    r = rnd(2, 96, 12, 10, seed=89)
    kw = dict(act="prelu", slope=sl, in_s=s_in, in_b=b_in, res=r, res_mode=mode, k_order=1, precision=2)
    got = run_conv(x, w, 1, 1, tile=tile, **kw)
    assert torch.equal(got, run_conv(x, w, 1, 1, tile=5, **kw))
    ref = ref_conv(x, w, 1, 1, act="prelu", slope=sl, in_s=s_in, in_b=b_in, res=r, res_mode=mode)
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-5)
    # stride-2 conv whose residual is a subsampled view of a full-resolution tensor
    big = rnd(2, 96, 12, 10, seed=90).permute(0, 2, 3, 1).contiguous().to(DEV)
    rview = big[:, ::2, ::2, :]
    pk = pack.pack_conv("t", w, 2, 1, DEV, k_order=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    outs = []
    for t in (tile, 5):
        y = torch.empty(2, 6, 5, 96, device=DEV)
        ops.conv2d(xd, pk, y, res=rview, res_mode=mode, precision=2, tile=t)
        outs.append(y.cpu())
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-6, atol=1e-6)
    ref2 = ref_conv(x, w, 2, 1, res=rview.cpu().permute(0, 3, 1, 2), res_mode=mode)
    torch.testing.assert_close(outs[0].permute(0, 3, 1, 2), ref2, rtol=0, atol=1e-5)


def _conv_p3(x, w, s, p, tile=0, amax=None, **kw):
    """precision 3 (split fp16, scaled): x_amax[n] = max|x[n]| per frame (or the given bound for
    every frame); returns (y, max over frames of y_amax) after checking y_amax[n] == max|y[n]|."""
    pk = pack.pack_conv("t", w, s, p, DEV, scale=kw.pop("scale", None), bias=kw.pop("bias", None),
                        act=kw.pop("act", "none"), k_order=1 if w.shape[2] * w.shape[3] > 1 else 0)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    B, _, H, W = x.shape
    Ho, Wo = (H + 2 * p - w.shape[2]) // s + 1, (W + 2 * p - w.shape[3]) // s + 1
    y = torch.empty(B, Ho, Wo, w.shape[0], device=DEV)
    xa = (frame_amax(x) if amax is None else torch.full((B,), float(amax))).to(DEV)
    ya = torch.zeros(B, device=DEV)
    r = kw.pop("res", None)
    rd = r.permute(0, 2, 3, 1).contiguous().to(DEV) if r is not None else None
    ops.conv2d(xd, pk, y, res=rd, precision=3, tile=tile, x_amax=xa, y_amax=ya, **kw)
    torch.cuda.synchronize()
    assert torch.equal(ya.cpu(), frame_amax(y))
    return y.permute(0, 3, 1, 2).cpu(), float(ya.max().item())


def frame_amax(t):
    """per-frame max|t| (the engine's y_amax slots), float32 CPU [B]"""
    return t.detach().abs().flatten(1).amax(1).float().cpu()


@pytest.mark.parametrize("tile", [0, 21, 22, 23, 24, 25, 26])
@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", WAVE_SHAPES)
def test_conv_f16_split_fp32_level_accuracy(B, Ci, H, W, Co, k, s, p, tile):
    """precision 3: per-output error vs fp64 within a few fp32 ulps of sum|x||w| (the CPU's own
    fp32 conv is the yardstick), far below the 2-plane bf16 split; y_amax == max|y| exactly."""
    x = torch.relu(rnd(B, Ci, H, W, seed=91)) * 7.0
    w = rnd(Co, Ci, k, k, seed=92, scale=1.0 / math.sqrt(Ci * k * k))
    sc = torch.rand(Co, generator=_g(93)) + 0.5
    bi = rnd(Co, seed=94)
    got, ymax = _conv_p3(x, w, s, p, tile=tile, scale=sc, bias=bi)
    ref = ref_conv(x, w, s, p, scale=sc, bias=bi).double()
    den = F.conv2d(x.double().abs(), w.double().abs(), None, s, p) * sc.double().view(1, -1, 1, 1)
    e16 = ((got.double() - ref).abs() / den).max().item()
    cpu = F.conv2d(x, w, None, s, p) * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1)
    e32 = ((cpu.double() - ref).abs() / den).max().item()
    bf = run_conv(x, w, s, p, scale=sc, bias=bi, precision=0, k_order=1 if k > 1 else 0)
    ebf = ((bf.double() - ref).abs() / den).max().item()
    f32 = run_conv(x, w, s, p, scale=sc, bias=bi, precision=2, k_order=1 if k > 1 else 0)
    e6 = ((f32.double() - ref).abs() / den).max().item()
    # the fp32-faithful 6-term mode and the CPU's fp32 conv are the yardsticks
    assert e16 <= max(3 * e6, 10 * e32, 2.0 ** -22), (e16, e6, e32)
    # far below the bf16 2-plane split, unless fp32 accumulation dominates both (K = 25088)
    assert e16 < ebf / 4 or e16 <= 1.5 * e6, (e16, ebf, e6)
    assert ymax == float(got.abs().max())


@pytest.mark.parametrize("amp", [1e-5, 1e-2, 1e2, 1e5])
def test_conv_f16_split_activation_scaling(amp):
    """The power-of-2 activation scale follows max|x| over 20 decades: no fp16 overflow at
    1e5, no lost low plane at 1e-5; a loose (larger) bound only costs low bits."""
    x = torch.relu(rnd(2, 64, 9, 11, seed=95)) * amp
    w = rnd(96, 64, 3, 3, seed=96, scale=0.05)
    ref = ref_conv(x, w, 1, 1).double()
    den = F.conv2d(x.double().abs(), w.double().abs(), None, 1, 1)
    for bound in (None, float(x.abs().max()) * 3.9):
        got, _ = _conv_p3(x, w, 1, 1, amax=bound)
        assert torch.isfinite(got).all()
        assert ((got.double() - ref).abs() / den).max().item() < 2 ** -20


def test_conv_f16_split_residual_and_chained_amax():
    """Producer -> consumer: the first conv's y_amax is the second's x_amax (the engine's
    wiring); residual + ReLU epilogue under precision 3."""
    x = rnd(2, 64, 10, 10, seed=97)
    w1 = rnd(128, 64, 1, 1, seed=98, scale=0.2)
    w2 = rnd(64, 128, 3, 3, seed=99, scale=0.03)
    r = rnd(2, 64, 10, 10, seed=100)
    p1 = pack.pack_conv("a", w1, 1, 0, DEV, act="relu")
    p2 = pack.pack_conv("b", w2, 1, 1, DEV, act="relu", k_order=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    xa = frame_amax(x).to(DEV)
    a1, a2 = torch.zeros(2, device=DEV), torch.zeros(2, device=DEV)
    t = torch.empty(2, 10, 10, 128, device=DEV)
    ops.conv2d(xd, p1, t, precision=3, x_amax=xa, y_amax=a1)
    y = torch.empty(2, 10, 10, 64, device=DEV)
    ops.conv2d(t, p2, y, res=r.permute(0, 2, 3, 1).contiguous().to(DEV), res_mode=RES_PRE, precision=3,
               x_amax=a1, y_amax=a2)
    torch.cuda.synchronize()
    assert torch.equal(a1.cpu(), frame_amax(t)) and torch.equal(a2.cpu(), frame_amax(y))
    ref = ref_conv(ref_conv(x, w1, 1, 0, act="relu"), w2, 1, 1, act="relu", res=r, res_mode=RES_PRE)
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=2e-6)


@pytest.mark.parametrize("precision", [0, 2, 3])
@pytest.mark.parametrize("stride,cin,c2,co", [(1, 64, 64, 256), (2, 128, 256, 512), (2, 64, 32, 96)])
def test_conv_dual_input_bottleneck_projection(precision, stride, cin, c2, co):
    """Dual-input 1x1 GEMM (ResNet block 0): relu(s3*(W3 o) + b3 + sd*(Wd x[::s, ::s]) + bd) with
    the BN scales folded into [W3 | Wd]; x2 is a subsampling view of the block input."""
    B, H, W = 2, 10, 12
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    o = torch.relu(rnd(B, cin, Ho, Wo, seed=106))
    xb = torch.relu(rnd(B, c2, H, W, seed=107))
    w3 = rnd(co, cin, 1, 1, seed=108, scale=0.1)
    wd = rnd(co, c2, 1, 1, seed=109, scale=0.1)
    s3, b3 = torch.rand(co, generator=_g(110)) + 0.5, rnd(co, seed=111)
    sd_, bd = torch.rand(co, generator=_g(112)) + 0.5, rnd(co, seed=113)
    w = torch.cat([w3.flatten(1) * s3[:, None], wd.flatten(1) * sd_[:, None]], 1)
    pk = pack.pack_matrix("d", w, 1, 1, cin + c2, 1, 0, DEV, bias=b3 + bd, act="relu")
    od = o.permute(0, 2, 3, 1).contiguous().to(DEV)
    xd = xb.permute(0, 2, 3, 1).contiguous().to(DEV)
    x2 = xd[:, ::stride, ::stride, :]
    y = torch.empty(B, Ho, Wo, co, device=DEV)
    amax = lambda t: frame_amax(t).to(DEV)
    ops.conv2d(od, pk, y, precision=precision, x2=x2, x_amax=amax(o), x2_amax=amax(xb))
    torch.cuda.synchronize()
    ref = torch.relu(ref_conv(o, w3, 1, 0, scale=s3, bias=b3).double() +
                     ref_conv(xb, wd, stride, 0, scale=sd_, bias=bd).double()).float()
    tol = 2e-4 if precision == 0 else 2e-6
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=tol)


def test_conv_dual_input_rejects_bad_geometry():
    o = rnd(1, 64, 5, 5, seed=114).permute(0, 2, 3, 1).contiguous().to(DEV)
    w = rnd(64, 96, 1, 1, seed=115)
    pk = pack.pack_conv("t", w, 1, 0, DEV)
    y = torch.empty(1, 5, 5, 64, device=DEV)
    with pytest.raises(PrpeError):                       # x2 not on the output grid
        ops.conv2d(o, pk, y, x2=torch.zeros(1, 6, 5, 32, device=DEV))
    with pytest.raises(PrpeError):                       # C2 % 32 != 0
        ops.conv2d(o, pack.pack_conv("t", rnd(64, 80, 1, 1, seed=116), 1, 0, DEV), y,
                   x2=torch.zeros(1, 5, 5, 16, device=DEV))


def _decode_planes(t):
    """planes format -> (hi, lo) fp32 tensors of the logical shape [N,H,W,C]."""
    n, h, w, c = t.shape
    u = t.contiguous().view(torch.int16).view(n, h, w, c // 8, 2, 8)
    hi = u[..., 0, :].contiguous().view(torch.bfloat16).float().reshape(n, h, w, c)
    lo = u[..., 1, :].contiguous().view(torch.bfloat16).float().reshape(n, h, w, c)
    return hi, lo


@pytest.mark.parametrize("k1,k2", [(1, 3), (3, 1), (3, 3)])
def test_planes_format_producer_consumer_bit_exact(k1, k2):
    """A conv writing the planes format + a precision-0 conv reading it == the fp32 tensor +
    the consumer's own split, bit for bit; the format holds hi = RNE(v), lo = RNE(v - hi)."""
    x = rnd(2, 64, 13, 11, seed=121).permute(0, 2, 3, 1).contiguous().to(DEV)
    w1 = rnd(128, 64, k1, k1, seed=122, scale=0.05)
    w2 = rnd(96, 128, k2, k2, seed=123, scale=0.03)
    p1 = pack.pack_conv("a", w1, 1, k1 // 2, DEV, act="silu")
    p2 = pack.pack_conv("b", w2, 1, k2 // 2, DEV, act="gelu")
    t32 = torch.empty(2, 13, 11, 128, device=DEV)
    tpl = torch.empty(2, 13, 11, 128, device=DEV)
    ops.conv2d(x, p1, t32, precision=0)
    ops.conv2d(x, p1, tpl, precision=0, y_planes=True)
    y32 = torch.empty(2, 13, 11, 96, device=DEV)
    ypl = torch.empty(2, 13, 11, 96, device=DEV)
    ops.conv2d(t32, p2, y32, precision=0, tile=26)
    ops.conv2d(tpl, p2, ypl, precision=0, x_planes=True)
    torch.cuda.synchronize()
    hi, lo = _decode_planes(tpl.cpu())
    v = t32.cpu()
    assert torch.equal(hi, v.to(torch.bfloat16).float())
    assert torch.equal(lo, (v - hi).to(torch.bfloat16).float())
    assert torch.equal(y32.cpu(), ypl.cpu())


@pytest.mark.parametrize("hi_,wi,ho,wo,act", [(20, 20, 160, 160, "silu"), (20, 20, 256, 192, "gelu")])
def test_upconv_planes_output_feeds_conv_bit_exact(hi_, wi, ho, wo, act):
    co = 64
    z = rnd(2, hi_, wi, 9 * co, seed=124).to(DEV)
    sc = (torch.rand(co, generator=_g(125)) + 0.5).to(DEV)
    bi = rnd(co, seed=126).to(DEV)
    u32 = torch.empty(2, ho, wo, co, device=DEV)
    upl = torch.empty(2, ho, wo, co, device=DEV)
    ops.upconv3x3(z, u32, True, sc, bi, None, act)
    ops.upconv3x3(z, upl, True, sc, bi, None, act, y_planes=True)
    w = rnd(128, co, 3, 3, seed=127, scale=0.05)
    pk = pack.pack_conv("c", w, 1, 1, DEV)
    y32 = torch.empty(2, ho, wo, 128, device=DEV)
    ypl = torch.empty(2, ho, wo, 128, device=DEV)
    ops.conv2d(u32, pk, y32, precision=0, tile=26)
    ops.conv2d(upl, pk, ypl, precision=0, x_planes=True)
    torch.cuda.synchronize()
    hi, lo = _decode_planes(upl.cpu())
    assert torch.equal(hi, u32.cpu().to(torch.bfloat16).float())
    assert torch.equal(y32.cpu(), ypl.cpu())


def test_layernorm_and_attention_planes_output_bit_exact():
    """LayerNorm / attention writing the planes format == their fp32 output split into
    hi = RNE(v), lo = RNE(v - hi) (the consumer GEMM's own split), bit for bit."""
    rows, c = 384, 768
    x = rnd(rows, c, seed=201, scale=3.0).to(DEV)
    g = (torch.rand(c, generator=_g(202)) + 0.5).to(DEV)
    b = rnd(c, seed=203).to(DEV)
    y32 = ops.layernorm(x, torch.empty(rows, c, device=DEV), g, b)
    ypl = ops.layernorm(x, torch.empty(rows, c, device=DEV), g, b, planes=True)
    B, L, H, D = 2, 192, 12, 64
    qkv = rnd(B * L, 3 * H * D, seed=204, scale=2.0).to(DEV)
    st = (L * 3 * H * D, H * D, D, 3 * H * D)
    o32 = ops.attention_strided(qkv, st, torch.empty(B * L, H * D, device=DEV), B, L, H, D, D ** -0.5)
    opl = ops.attention_strided(qkv, st, torch.empty(B * L, H * D, device=DEV), B, L, H, D, D ** -0.5,
                                out_planes=True)
    torch.cuda.synchronize()
    for v32, vpl in ((y32, ypl), (o32, opl)):
        n = v32.shape[0]
        hi, lo = _decode_planes(vpl.cpu().view(n, 1, 1, -1))
        v = v32.cpu().view(n, 1, 1, -1)
        assert torch.equal(hi, v.to(torch.bfloat16).float())
        assert torch.equal(lo, (v - hi).to(torch.bfloat16).float())


def test_planes_format_rejected_outside_precision_0():
    x = rnd(1, 64, 5, 5, seed=128).permute(0, 2, 3, 1).contiguous().to(DEV)
    pk = pack.pack_conv("t", rnd(64, 64, 1, 1, seed=129), 1, 0, DEV)
    y = torch.empty(1, 5, 5, 64, device=DEV)
    with pytest.raises(PrpeError):
        ops.conv2d(x, pk, y, precision=2, x_planes=True)


def test_conv_y_amax_every_kernel_family():
    """y_amax from the register-staged (scalar and vector epilogues), LDS-DMA and wave-row
    kernels and the small-Co kernel."""
    x = rnd(2, 64, 9, 13, seed=101)
    for co, tile, k in ((150, 5, 3), (152, 5, 3), (152, 10, 3), (152, 21, 3), (3, 0, 1)):
        w = rnd(co, 64, k, k, seed=102, scale=0.05)
        pk = pack.pack_conv("t", w, 1, k // 2, DEV, k_order=1 if k > 1 else 0)
        xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
        y = torch.empty(2, 9, 13, co, device=DEV)
        ya = torch.zeros(2, device=DEV)
        ops.conv2d(xd, pk, y, precision=2, tile=tile, y_amax=ya)
        torch.cuda.synchronize()
        assert torch.equal(ya.cpu(), frame_amax(y)), (co, tile)


def test_conv_fp32_faithful_stem_scalar_path():
    x = rnd(2, 3, 48, 48, seed=48)
    w = rnd(64, 3, 7, 7, seed=49, scale=0.1)
    got = run_conv(x, w, 2, 3, precision=2, x_layout="nchw")
    ref = ref_conv(x, w, 2, 3)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-6)


@pytest.mark.parametrize("hi,wi,ho,wo,ac,act", [(20, 20, 160, 160, True, "silu"), (20, 20, 112, 112, True, "prelu"),
                                               (20, 20, 256, 192, True, "gelu"), (16, 12, 64, 48, False, "none")])
@pytest.mark.parametrize("separable", [True, False])
def test_upconv_equals_upsample_then_conv(hi, wi, ho, wo, ac, act, separable):
    Ci, Co = 32, 24
    x = rnd(2, Ci, hi, wi, seed=23)
    w = rnd(Co, Ci, 3, 3, seed=24, scale=0.05)
    sc = torch.rand(Co, generator=_g(25)) + 0.5
    bi = rnd(Co, seed=26)
    sl = torch.rand(Co, generator=_g(27)) * 0.4
    taps = pack.pack_upconv_taps("t", w, DEV)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    z = torch.empty(2, hi, wi, 9 * Co, device=DEV)
    ops.conv2d(xd, taps, z)
    y = torch.empty(2, ho, wo, Co, device=DEV)
    ops.upconv3x3(z, y, ac, sc.to(DEV), bi.to(DEV), sl.to(DEV) if act == "prelu" else None, act,
                  separable=separable)
    torch.cuda.synchronize()
    u = F.interpolate(x.double(), size=(ho, wo), mode="bilinear", align_corners=ac)
    ref = F.conv2d(u, w.double(), None, 1, 1) * sc.double().view(1, -1, 1, 1) + bi.double().view(1, -1, 1, 1)
    ref = act_ref(ref.float(), act, sl)
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=2e-4)


@pytest.mark.parametrize("h,w,ci,co,act", [(256, 192, 128, 3, "gelu"), (160, 160, 64, 3, "silu"),
                                         (7, 5, 32, 1, "none"), (1, 1, 64, 4, "silu"), (13, 29, 96, 2, "gelu")])
def test_conv3x3_smallco_tap_rewrite(h, w, ci, co, act):
    """Engine.conv3x3_smallco: a 3x3/1 pad-1 conv with Co <= 4 as the 1x1 tap GEMM plus the
    unit-scale tap sum of prpe_upconv3x3 (align_corners=True, output grid = input grid, so
    every source index is exact). Against the direct conv in fp64; tolerance as the other
    split-bf16 convs (2e-4 abs on O(1) data, K = 9*ci)."""
    x = rnd(2, ci, h, w, seed=230)
    wt = rnd(co, ci, 3, 3, seed=231, scale=0.05)
    sc = torch.rand(co, generator=_g(232)) + 0.5
    bi = rnd(co, seed=233)
    taps = pack.pack_upconv_taps("t", wt, DEV)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    z = torch.empty(2, h, w, 9 * co, device=DEV)
    ops.conv2d(xd, taps, z)
    y = torch.empty(2, h, w, co, device=DEV)
    ops.upconv3x3(z, y, True, sc.to(DEV), bi.to(DEV), None, act)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double(), wt.double(), None, 1, 1) * sc.double().view(1, -1, 1, 1) + bi.double().view(1, -1, 1, 1)
    ref = act_ref(ref.float(), act)
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=2e-4)


@pytest.mark.parametrize("co", [1, 3, 4])
@pytest.mark.parametrize("act", ["gelu", "silu", "prelu"])
def test_upconv_unit_scale_tap_sum_bit_exact(co, act):
    """The unit-scale upconv (output grid = input grid, align_corners; round 6's tap-sum kernel for
    Co <= 4) == the two-pass separable form bit for bit, incl. an NHWC4-strided output view (the
    4th channel untouched), and its per-frame max|y| slots."""
    h, w = 37, 53
    z = rnd(2, h, w, 9 * co, seed=240, scale=2.0).to(DEV)
    sc = (torch.rand(co, generator=_g(241)) + 0.5).to(DEV)
    bi = rnd(co, seed=242).to(DEV)
    sl = (torch.rand(co, generator=_g(243)) * 0.3).to(DEV) if act == "prelu" else None
    ref = torch.empty(2, h, w, co, device=DEV)
    ops.upconv3x3(z, ref, True, sc, bi, sl, act, separable=True)
    y = torch.empty(2, h, w, co, device=DEV)
    ya = torch.zeros(2, device=DEV)
    ops.upconv3x3(z, y, True, sc, bi, sl, act, y_amax=ya)
    buf = torch.full((2, h, w, 4), 7.0, device=DEV)
    ops.upconv3x3(z, buf[..., :co], True, sc, bi, sl, act)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), ref.cpu())
    assert torch.equal(buf[..., :co].cpu(), ref.cpu())
    assert torch.equal(buf[..., co:].cpu(), torch.full_like(buf[..., co:].cpu(), 7.0))
    assert torch.equal(ya.cpu(), ref.abs().amax(dim=(1, 2, 3)).cpu())


@pytest.mark.parametrize("act", ["silu", "sigmoid", "gelu", "relu"])
def test_epilogue_activation_accuracy(act):
    """apply_act (every conv / upconv epilogue; SiLU and sigmoid on the hardware exp2 with a
    two-part argument) against fp64 torch or the fp32 CPU result: within 4 ulp of either plus
    1e-35 absolute (where exp(-v) overflows fp32 every fp32 form, the CPU one included, gives
    -0 for values of order -1e-37), and no NaN at overflow (|v| up to 1e4). Driven through
    prpe_upconv3x3 at unit scale with only the centre tap non-zero, so the epilogue sees v
    exactly."""
    v = torch.cat([torch.linspace(-120, 120, 4801), torch.tensor([0.0, -0.0, 1e-30, -1e-30, 88.7, -88.7, 89.5,
                                                                   -89.5, 104.0, -104.0, 1e4, -1e4, 1e-3, -1e-3])])
    n = v.numel()
    W = 64
    H = (n + W - 1) // W
    x = torch.zeros(H * W)
    x[:n] = v
    z = torch.zeros(1, H, W, 9 * 4)
    z[0, :, :, 4 * 4] = x.view(H, W)           # tap (dy=1, dx=1), channel 0
    y = torch.empty(1, H, W, 4, device=DEV)
    ops.upconv3x3(z.to(DEV), y, True, torch.ones(4, device=DEV), torch.zeros(4, device=DEV), None, act)
    torch.cuda.synchronize()
    got = y[0, :, :, 0].reshape(-1)[:n].cpu().double()
    vd = v.double()
    ref = {"silu": vd * torch.sigmoid(vd), "sigmoid": torch.sigmoid(vd), "gelu": F.gelu(vd),
           "relu": F.relu(vd)}[act]
    # the CPU reference's own fp32 arithmetic (GELU's 1 + erf cancels below v ~ -5 there too)
    ref32 = {"silu": F.silu(v), "sigmoid": torch.sigmoid(v), "gelu": F.gelu(v), "relu": F.relu(v)}[act].double()
    assert not torch.isnan(got).any()
    ulp = torch.finfo(torch.float32).eps * ref.float().double().abs()
    # GELU: 0.5 v (1 + erf(v / sqrt 2)) inherits erf's absolute rounding (2^-24) times |v|
    tol = 4 * ulp + 1e-35 + (2.0 ** -22 * vd.abs() if act == "gelu" else 0.0)
    bad = ((got - ref).abs() > tol) & ((got - ref32).abs() > tol)
    assert not bad.any(), (v[bad][:8], got[bad][:8], ref[bad][:8])


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["silu", "sigmoid", "gelu"])
def test_epilogue_activation_inf_nan(act):
    """apply_act at +-inf and NaN. GELU (single-branch form, common.h gelu_v): +inf -> +inf and
    -inf -> 0, the activation's limits (torch's CPU GELU gives NaN at both). Every activation keeps
    a NaN a NaN. SiLU / sigmoid at +-inf are NaN here by design: exp_hw's two-part argument
    (x log2 e = t + e) is inf - inf there, and guarding it would add VALU to the VALU-bound upconv
    epilogues for inputs the model never produces (its pre-activations are finite). Each special
    value sits on its own pixel with zero neighbours (at unit scale the bilinear weights of the
    neighbours are 0, and 0 * inf would make THEM NaN -- a property of the harness, not of the
    epilogue)."""
    vals = [float("inf"), float("-inf"), float("nan")]
    H = W = 8
    z = torch.zeros(1, H, W, 9 * 4)
    pos = [(1, 1), (1, 4), (4, 1)]
    for (i, j), v in zip(pos, vals):
        z[0, i, j, 4 * 4] = v                   # tap (dy=1, dx=1), channel 0
    y = torch.empty(1, H, W, 4, device=DEV)
    ops.upconv3x3(z.to(DEV), y, True, torch.ones(4, device=DEV), torch.zeros(4, device=DEV), None, act)
    torch.cuda.synchronize()
    got = [y[0, i, j, 0].item() for i, j in pos]
    if act == "gelu":
        assert got[0] == math.inf and got[1] == 0.0, got
    assert math.isnan(got[2]), got


@pytest.mark.parametrize("hi,wi,ho,wo,ac", [(20, 20, 160, 160, True), (20, 20, 256, 192, True),
                                        (16, 12, 64, 48, False), (7, 9, 20, 13, False), (20, 20, 23, 21, True),
                                        (20, 20, 112, 112, True), (9, 5, 40, 17, False), (13, 6, 37, 11, True),
                                        (20, 7, 51, 9, False), (11, 4, 61, 8, True)])
@pytest.mark.parametrize("Co", [24, 64])
def test_upconv_fused_matches_separable(hi, wi, ho, wo, ac, Co):
    """The one-pass kernels (rolling-row; LDS-DMA where Co % 32 == 0 and the ratio is >= 5, i.e.
    Co = 64 at the adapters' ratios) and the two-pass separable form evaluate the same sum in
    the same rounding sequence (pointwise.hip lerp_add): bit-identical, at the adapters'
    upsampling ratios and at awkward ones (source intervals of 1-2 output rows, both
    align_corners modes)."""
    z = rnd(2, hi, wi, 9 * Co, seed=103).to(DEV)
    sc = (torch.rand(Co, generator=_g(104)) + 0.5).to(DEV)
    bi = rnd(Co, seed=105).to(DEV)
    outs = []
    for sep in (False, True):
        y = torch.empty(2, ho, wo, Co, device=DEV)
        ops.upconv3x3(z, y, ac, sc, bi, None, "gelu", separable=sep)
        outs.append(y.cpu())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("hi,wi,ho,wo,co,act", [(20, 20, 160, 160, 512, "silu"), (20, 20, 256, 192, 256, "gelu"),
                                              (20, 20, 112, 112, 256, "prelu"), (20, 20, 100, 70, 96, "none")])
@pytest.mark.parametrize("planes", [False, True])
def test_upconv_dma_kernel_model_shapes_bit_exact(hi, wi, ho, wo, co, act, planes):
    """The LDS-DMA upconv (the adapters' shapes: face-YOLO 20->160 Co 512, ViTPose 20->256x192
    Co 256, AdaFace 20->112 Co 256, and a ragged column tile) == the separable form bit for bit,
    fp32 output and planes output (hi = RNE(v), lo = RNE(v - hi) of the same values)."""
    z = rnd(2, hi, wi, 9 * co, seed=128).to(DEV)
    sc = (torch.rand(co, generator=_g(129)) + 0.5).to(DEV)
    bi = rnd(co, seed=130).to(DEV)
    sl = (torch.rand(co, generator=_g(131)) * 0.3).to(DEV) if act == "prelu" else None
    ref = torch.empty(2, ho, wo, co, device=DEV)
    ops.upconv3x3(z, ref, True, sc, bi, sl, act, separable=True)
    y = torch.empty(2, ho, wo, co, device=DEV)
    ops.upconv3x3(z, y, True, sc, bi, sl, act, y_planes=planes)
    torch.cuda.synchronize()
    if planes:
        h, l = _decode_planes(y.cpu())
        v = ref.cpu()
        assert torch.equal(h, v.to(torch.bfloat16).float())
        assert torch.equal(l, (v - h).to(torch.bfloat16).float())
    else:
        assert torch.equal(y.cpu(), ref.cpu())


def test_upconv_nchw_output_view():
    x = rnd(1, 16, 16, 12, seed=28)
    w = rnd(17, 16, 3, 3, seed=29, scale=0.1)
    bi = rnd(17, seed=30)
    taps = pack.pack_upconv_taps("t", w, DEV)
    z = torch.empty(1, 16, 12, 9 * 17, device=DEV)
    ops.conv2d(x.permute(0, 2, 3, 1).contiguous().to(DEV), taps, z)
    heat = torch.empty(1, 17, 64, 48, device=DEV)
    ops.upconv3x3(z, ops.nhwc(heat), False, None, bi.to(DEV), None, "none")
    torch.cuda.synchronize()
    ref = F.conv2d(F.interpolate(x, scale_factor=4.0, mode="bilinear", align_corners=False), w, bi, 1, 1)
    torch.testing.assert_close(heat.cpu(), ref, rtol=0, atol=1e-4)


def test_dwconv_with_residual():
    x = rnd(2, 80, 10, 10, seed=31)
    w = rnd(80, 1, 3, 3, seed=32)
    sc = torch.rand(80, generator=_g(33)) + 0.5
    bi = rnd(80, seed=34)
    r = rnd(2, 80, 10, 10, seed=35)
    y = torch.empty(2, 10, 10, 80, device=DEV)
    ops.dwconv(x.permute(0, 2, 3, 1).contiguous().to(DEV), y, w.reshape(-1).to(DEV), 3, 1, 1, sc.to(DEV), bi.to(DEV),
               "silu", res=r.permute(0, 2, 3, 1).contiguous().to(DEV))
    torch.cuda.synchronize()
    ref = F.silu(F.conv2d(x, w, None, 1, 1, 1, 80) * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1)) + r
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=1e-5)


@pytest.mark.parametrize("k,s,p,H", [(3, 2, 1, 33), (5, 1, 2, 5), (1, 2, 0, 14)])
def test_maxpool(k, s, p, H):
    x = rnd(2, 16, H, H, seed=36)
    Ho = (H + 2 * p - k) // s + 1
    y = torch.empty(2, Ho, Ho, 16, device=DEV)
    ops.maxpool(x.permute(0, 2, 3, 1).contiguous().to(DEV), y, k, s, p)
    torch.cuda.synchronize()
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), F.max_pool2d(x, k, s, p), rtol=0, atol=0)


def test_upsample_nearest2x():
    x = rnd(2, 8, 5, 5, seed=37)
    y = torch.empty(2, 10, 10, 8, device=DEV)
    ops.upsample_nearest2x(x.permute(0, 2, 3, 1).contiguous().to(DEV), y)
    torch.cuda.synchronize()
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), F.interpolate(x, scale_factor=2.0, mode="nearest"),
                               rtol=0, atol=0)


@pytest.mark.parametrize("B,C,H,W,nchw_out", [(2, 3, 160, 160, False), (2, 1, 3, 1100, True), (1, 4, 33, 31, True),
                                              (2, 2, 1, 2, False)])
def test_norm_sigmoid_shapes(B, C, H, W, nchw_out):
    """Per-sample per-channel standardisation + sigmoid (modify_models.py:84-86) at the model's
    160x160, rows wider than one block (W > 1024), ragged sizes, C = 1..4, NCHW output view."""
    x = rnd(B, C, H, W, seed=39, scale=3.0) + 0.7
    if nchw_out:
        yb = torch.empty(B, C, H, W, device=DEV)
        y = yb.permute(0, 2, 3, 1)
    else:
        y = torch.empty(B, H, W, C, device=DEV)
    ops.norm_sigmoid(x.permute(0, 2, 3, 1).contiguous().to(DEV), y)
    torch.cuda.synchronize()
    r = x.double() - x.double().mean(dim=(2, 3), keepdim=True)
    r = torch.sigmoid(r / (r.std(dim=(2, 3), keepdim=True) + 1e-6)).float()
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), r, rtol=0, atol=2e-6)


def test_norm_sigmoid():
    x = rnd(3, 3, 40, 40, seed=38, scale=3.0) + 0.7
    y = torch.empty(3, 40, 40, 3, device=DEV)
    ops.norm_sigmoid(x.permute(0, 2, 3, 1).contiguous().to(DEV), y)
    torch.cuda.synchronize()
    r = x - x.mean(dim=(2, 3), keepdim=True)
    r = torch.sigmoid(r / (r.std(dim=(2, 3), keepdim=True) + 1e-6))
    torch.testing.assert_close(y.permute(0, 3, 1, 2).cpu(), r, rtol=0, atol=2e-6)


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("C", [768, 200, 1000, 770])
def test_layernorm(relu, C):
    """register-resident kernel (C % 4 == 0, C <= 1024) and the generic one (C = 770)"""
    x = rnd(384, C, seed=39, scale=4.0) + 1.0
    g = torch.rand(C, generator=_g(40)) + 0.5
    b = rnd(C, seed=41)
    y = torch.empty(384, C, device=DEV)
    ops.layernorm(x.to(DEV), y, g.to(DEV), b.to(DEV), 1e-12, relu)
    torch.cuda.synchronize()
    ref = F.layer_norm(x, (C,), g, b, 1e-12)
    if relu:
        ref = F.relu(ref)
    torch.testing.assert_close(y.cpu(), ref, rtol=0, atol=1e-5)


def test_vit_attention():
    B, L, H, D = 3, 192, 12, 64
    qkv = rnd(B * L, 3 * H * D, seed=42, scale=2.0)
    out = torch.empty(B * L, H * D, device=DEV)
    ops.attention(qkv.to(DEV), out, B, L, H, D, D ** -0.5)
    torch.cuda.synchronize()
    q, k, v = qkv.view(B, L, 3, H, D).permute(2, 0, 3, 1, 4).double()
    att = torch.softmax(q @ k.transpose(-1, -2) * D ** -0.5, -1)
    ref = (att @ v).transpose(1, 2).reshape(B * L, H * D).float()
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=5e-5)


def test_vit_attention_online_softmax_rescale():
    # one key per chunk region made dominant for chosen queries, so the running max jumps in a
    # late key chunk (the O / l rescale branch is taken with a large factor), plus a query whose
    # logits are all equal (uniform weights)
    B, L, H, D = 2, 192, 12, 64
    qkv = rnd(B * L, 3 * H * D, seed=44, scale=1.0).view(B, L, 3, H, D)
    for q, key in ((5, 170), (40, 3), (100, 65), (191, 191)):
        qkv[0, key, 1, 2] = 4.0 * qkv[0, q, 0, 2]        # frame 0, head 2: q . k large
    qkv[1, 7, 0, 5] = 0.0                                 # frame 1, head 5, query 7: all logits 0
    qkv = qkv.reshape(B * L, 3 * H * D)
    out = torch.empty(B * L, H * D, device=DEV)
    ops.attention(qkv.to(DEV), out, B, L, H, D, D ** -0.5)
    torch.cuda.synchronize()
    q, k, v = qkv.view(B, L, 3, H, D).permute(2, 0, 3, 1, 4).double()
    att = torch.softmax(q @ k.transpose(-1, -2) * D ** -0.5, -1)
    ref = (att @ v).transpose(1, 2).reshape(B * L, H * D).float()
    torch.testing.assert_close(out.cpu(), ref, rtol=0, atol=5e-5)


def test_vit_attention_head_major_operand_bit_identical():
    B, L, H, D = 2, 192, 12, 64
    qkv = rnd(B * L, 3 * H * D, seed=45, scale=2.0).to(DEV)
    a = torch.empty(B * L, H * D, device=DEV)
    b = torch.empty(B * L, H * D, device=DEV)
    ops.attention(qkv, a, B, L, H, D, D ** -0.5)
    hm = qkv.view(B, L, 3, H, D).permute(0, 2, 3, 1, 4).contiguous()
    ops.attention_strided(hm, (3 * H * L * D, H * L * D, L * D, D), b, B, L, H, D, D ** -0.5)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("B", [4, 1232])
def test_vit_attention_frame_interleaved_operand(B):
    """a frame-interleaved [L, B, 3, H, D] operand (s_tok = B * 3HD). At B = 4 the
    frame's extent fits the whole-head kernel's 32-bit buffer offsets (bit-identical to the
    row-major call); at B = 1232 it spans > 2^31 bytes and must be routed to the 64-bit streaming
    kernel instead of silently reading zeros (checked against fp64 on spread frames)."""
    L, H, D = 192, 12, 64
    qkv = rnd(B * L, 3 * H * D, seed=46, scale=2.0).to(DEV)
    a = torch.empty(B * L, H * D, device=DEV)
    ops.attention(qkv, a, B, L, H, D, D ** -0.5)
    il = qkv.view(B, L, 3 * H * D).transpose(0, 1).contiguous()          # [L, B, 3HD]
    st = (3 * H * D, H * D, D, B * 3 * H * D)
    assert ((L - 1) * st[3] + 2 * st[1] + (H - 1) * st[2] + D) * 4 >= (1 << 31) or B < 1000
    b = torch.empty(B * L, H * D, device=DEV)
    ops.attention_strided(il, st, b, B, L, H, D, D ** -0.5)
    torch.cuda.synchronize()
    if B < 1000:
        assert torch.equal(a, b)
        return
    del il
    ac, bc = a.cpu(), b.cpu()
    for f in (0, B // 2, B - 1):
        q, k, v = qkv[f * L:(f + 1) * L].cpu().view(L, 3, H, D).permute(1, 2, 0, 3).double()
        ref = (torch.softmax(q @ k.transpose(-1, -2) * D ** -0.5, -1) @ v).transpose(0, 1).reshape(L, H * D)
        torch.testing.assert_close(bc[f * L:(f + 1) * L], ref.float(), rtol=0, atol=5e-5)
    torch.testing.assert_close(bc, ac, rtol=0, atol=1e-4)    # two kernels, each within 5e-5 of fp64


def test_vit_attention_negative_stride_rejected():
    B, L, H, D = 2, 192, 12, 64
    qkv = rnd(B * L, 3 * H * D, seed=47).to(DEV)
    out = torch.empty(B * L, H * D, device=DEV)
    with pytest.raises(PrpeError):
        ops.attention_strided(qkv, (L * 3 * H * D, H * D, D, -3 * H * D), out, B, L, H, D, D ** -0.5)


@pytest.mark.parametrize("hw", [5, 20, 17])
def test_psa_attention(hw):
    """5x5: the LDS score-matrix kernel (the model's P5 after the adapter); 20x20 (raw 640x640
    frames, the config-2 micro-bench variant) and 17x17: the streaming two-pass kernel."""
    B, nh, dk, dh = 2, 2, 32, 64
    per = 2 * dk + dh
    L = hw * hw
    qkv = rnd(B, nh * per, hw, hw, seed=43, scale=2.0)
    out = torch.empty(B, hw, hw, nh * dh, device=DEV)
    vout = torch.empty(B, hw, hw, nh * dh, device=DEV)
    ops.psa_attention(qkv.permute(0, 2, 3, 1).contiguous().to(DEV), out, vout, nh, dk, dh, dk ** -0.5)
    torch.cuda.synchronize()
    t = qkv.view(B, nh, per, L).double()
    q, k, v = t.split([dk, dk, dh], dim=2)
    att = ((q.transpose(-2, -1) @ k) * dk ** -0.5).softmax(-1)
    ref = (v @ att.transpose(-2, -1)).reshape(B, nh * dh, hw, hw).float()
    torch.testing.assert_close(out.permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=1e-5)
    torch.testing.assert_close(vout.permute(0, 3, 1, 2).cpu(), v.float().reshape(B, nh * dh, hw, hw), rtol=0, atol=0)


def test_l2norm():
    x = rnd(37, 512, seed=44, scale=5.0)
    emb = torch.empty(37, 512, device=DEV)
    nrm = torch.empty(37, 1, device=DEV)
    ops.l2norm(x.to(DEV), emb, nrm)
    torch.cuda.synchronize()
    n = torch.norm(x, 2, 1, True)
    torch.testing.assert_close(nrm.cpu(), n, rtol=1e-6, atol=0)
    torch.testing.assert_close(emb.cpu(), x / n, rtol=0, atol=1e-7)


def test_l2norm_zero_rows_eps():
    """eps = 1e-12 is F.normalize (a zero row stays 0, face-rec eval); eps = 0 is the IR-50
    output's torch.div(x, norm) (a zero row gives NaN there too)."""
    x = rnd(8, 512, seed=46)
    x[3] = 0.0
    x[5] *= 1e-20                               # norm below eps: x / 1e-12
    xd = x.to(DEV)
    emb, nrm = torch.empty(8, 512, device=DEV), torch.empty(8, 1, device=DEV)
    ops.l2norm(xd, emb, nrm, 1e-12)
    torch.cuda.synchronize()
    ref = torch.nn.functional.normalize(x)
    torch.testing.assert_close(emb.cpu(), ref, rtol=1e-6, atol=1e-7)
    assert torch.equal(emb[3].cpu(), torch.zeros(512)) and nrm[3].item() == 0.0
    ops.l2norm(xd, emb, nrm, 0.0)
    torch.cuda.synchronize()
    ref0 = torch.div(x, torch.norm(x, 2, 1, True))
    assert torch.isnan(emb[3]).all() and torch.isnan(ref0[3]).all()
    ok = torch.arange(8) != 3
    torch.testing.assert_close(emb.cpu()[ok], ref0[ok], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("stride", [(0.0, 0.0, 0.0), (8.0, 16.0, 32.0)])
def test_dfl_decode_matches_oracle_head(stride):
    from oracle.model_ref import make_anchors
    B, A = 2, 525
    head = rnd(B, A, 65, seed=45, scale=3.0)
    det = torch.empty(B, 5, A, device=DEV)
    ops.dfl_decode(head.to(DEV), det, 1, [(20, 20), (10, 10), (5, 5)], stride)
    torch.cuda.synchronize()
    # oracle decode (nn.py:261-270)
    feats = [torch.zeros(B, 65, h, h) for h in (20, 10, 5)]
    anchors, strides = (t.transpose(0, 1) for t in make_anchors(feats, stride))
    x = head.transpose(1, 2)
    box, cls = x.split((64, 1), 1)
    d = box.reshape(B, 4, 16, A).transpose(2, 1).softmax(1)
    d = F.conv2d(d, torch.arange(16, dtype=torch.float32).view(1, 16, 1, 1)).view(B, 4, A)
    lt, rb = d.chunk(2, 1)
    a1, b1 = anchors.unsqueeze(0) - lt, anchors.unsqueeze(0) + rb
    ref = torch.cat((torch.cat(((a1 + b1) / 2, b1 - a1), 1) * strides, cls.sigmoid()), 1)
    torch.testing.assert_close(det.cpu(), ref, rtol=2e-6, atol=2e-5)


@pytest.mark.parametrize("yc,flip", [(4, False), (4, True), (5, False), (8, True)])
def test_copy_pad_nchw_to_padded_nhwc(yc, flip):
    """prpe_copy_pad: NCHW frames (read in place through a permuted view) into the interior of a
    zero-bordered NHWC buffer with yc >= 3 channels (4 = the stem's NHWC4 buffer: one 16-B
    store per pixel), optionally mirrored along W, raising max|y|. Exact copy."""
    x = torch.randn(2, 3, 13, 21)
    buf = torch.full((2, 13 + 6, 21 + 8, yc), 7.0, device=DEV)
    y = buf[:, 3:3 + 13, 4:4 + 21, :]
    ya = torch.zeros(2, device=DEV)
    ops.copy_pad(x.to(DEV).permute(0, 2, 3, 1), y, flip_w=flip, y_amax=ya)
    torch.cuda.synchronize()
    ref = x.flip(3) if flip else x
    got = y.cpu()
    assert torch.equal(got[..., :3], ref.permute(0, 2, 3, 1))
    assert torch.equal(got[..., 3:], torch.zeros_like(got[..., 3:]))
    assert torch.equal(ya.cpu(), frame_amax(x))                # per-frame max|y|
    # the border is untouched
    assert torch.equal(buf[:, :3].cpu(), torch.full_like(buf[:, :3].cpu(), 7.0))
