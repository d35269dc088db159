"""GPU: precision 4 (ONE scaled fp16 plane per operand, one MFMA per product; the AdaFace
branch's policy, engine.AUTO_POLICY) in the wave-row and haloed-tile conv kernels, and the
per-frame max|y| output of prpe_upconv3x3 that feeds it.

The kernels are checked against a CPU emulation of the declared operand rounding (prpe.h,
``precision``): w_eff = RNE_fp16(w 2^e[co]) 2^-e[co] (the pack's hi plane), x_eff =
RNE_fp16(x 2^s[n]) 2^-s[n] with s[n] = 15 - e(x_amax[n]) (for a prologue conv, of the bound
x_amax max|in_scale| + max|in_bias|), products summed in fp64. Against that emulation only fp32
accumulation remains: |d| <= 1e-5 sum|x_eff||w_eff| (fp32 over K <= 4608 terms is ~1e-6). Against
exact fp64 the declared operand error holds: |d| <= 2^-10 sum|x||w| (two RNE roundings of 2^-12).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from prpe import ops, pack
from prpe._lib import RES_PRE

from test_gpu_ops import DEV, _g, frame_amax, ref_conv, rnd

pytestmark = pytest.mark.gpu


def _f16_exp(m):
    """f16_scale_exp (common.h): m < 2^e, e = 15 for m == 0"""
    _, e = torch.frexp(m)
    return torch.where(m > 0, e, torch.full_like(e, 15))


def _w_eff(w):
    """the pack's hi fp16 plane, rescaled: RNE(w 2^e[co]) 2^-e[co] (pack.split_f16_scaled)"""
    w2 = w.reshape(w.shape[0], -1).float()
    m = w2.abs().amax(1)
    _, ex = torch.frexp(m)
    e = torch.where(m > 0, 15 - ex, torch.zeros_like(ex))
    hi = torch.ldexp(w2, e.view(-1, 1)).half().float()
    return torch.ldexp(hi, -e.view(-1, 1)).view_as(w)


def _x_eff(x, bound):
    """x [B, C, H, W] -> RNE_fp16(x 2^s[n]) 2^-s[n], s[n] = 15 - e(bound[n])"""
    s = (15 - _f16_exp(bound)).view(-1, 1, 1, 1)
    return torch.ldexp(torch.ldexp(x.float(), s).half().float(), -s)


def _conv_p4(x, w, s, p, tile=0, in_s=None, in_b=None, res=None, res_mode=0, act="none", scale=None,
             bias=None, slope=None, bound=None):
    pk = pack.pack_conv("p4", w, s, p, DEV, scale=scale, bias=bias, slope=slope, in_scale=in_s, in_bias=in_b,
                        act=act, k_order=1 if w.shape[2] * w.shape[3] > 1 else 0)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    B, _, H, W = x.shape
    Ho, Wo = (H + 2 * p - w.shape[2]) // s + 1, (W + 2 * p - w.shape[3]) // s + 1
    y = torch.empty(B, Ho, Wo, w.shape[0], device=DEV)
    xa = (frame_amax(x) if bound is None else bound).to(DEV)
    ya = torch.zeros(B, device=DEV)
    rd = res.permute(0, 2, 3, 1).contiguous().to(DEV) if res is not None else None
    ops.conv2d(xd, pk, y, res=rd, res_mode=res_mode, precision=4, tile=tile, x_amax=xa, y_amax=ya)
    torch.cuda.synchronize()
    got = y.permute(0, 3, 1, 2).cpu()
    assert torch.equal(ya.cpu(), frame_amax(got)), "y_amax must be max|y| per frame"
    return got


def _emul(x, w, s, p, xa, in_s=None, in_b=None, scale=None, bias=None, act="none", slope=None, res=None,
          res_mode=0):
    """fp64 conv of the precision-4 operands (see module docstring) + the epilogue"""
    xx = x.float()
    bound = xa.clone()
    if in_s is not None:
        xx = xx * in_s.view(1, -1, 1, 1) + in_b.view(1, -1, 1, 1)
        bound = xa * in_s.abs().max() + in_b.abs().max()
    xe = _x_eff(xx, bound)                         # padding taps are zero after the prologue
    we = _w_eff(w)
    v = F.conv2d(xe.double(), we.double(), None, s, p)
    den = F.conv2d(xe.double().abs(), we.double().abs(), None, s, p)
    sc = scale.double().view(1, -1, 1, 1) if scale is not None else 1.0
    v = v * sc
    den = den * (scale.double().abs().view(1, -1, 1, 1) if scale is not None else 1.0)
    if bias is not None:
        v = v + bias.double().view(1, -1, 1, 1)
    if res_mode == RES_PRE:
        v = v + res.double()
    if act == "prelu":
        v = F.prelu(v, slope.double())
    elif act == "relu":
        v = F.relu(v)
    elif act != "none":
        v = {"silu": F.silu, "gelu": F.gelu}[act](v)
    return v, den


P4_SHAPES = [
    (2, 64, 17, 19, 96, 3, 1, 1),       # ragged spatial / Co
    (2, 128, 11, 9, 64, 3, 2, 1),       # 3x3 / 2 (IR-50 res4 of a downsampling unit)
    (2, 64, 20, 20, 256, 1, 1, 0),      # 1x1 (the adapter's tap GEMM)
    (1, 256, 10, 10, 512, 1, 2, 0),     # 1x1 / 2 (IR-50 shortcut)
    (3, 96, 13, 17, 136, 3, 1, 1),      # Co beyond one 128 tile
    (2, 256, 14, 14, 256, 3, 1, 1),     # IR-50 body.8 shape
]


@pytest.mark.parametrize("tile", [0, 24, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("B,Ci,H,W,Co,k,s,p", P4_SHAPES)
def test_conv_p4_matches_operand_emulation(B, Ci, H, W, Co, k, s, p, tile):
    x = torch.relu(rnd(B, Ci, H, W, seed=401)) * 7.0
    x[1:] *= 0.01                                   # frames of very different scale: per-frame s[n]
    w = rnd(Co, Ci, k, k, seed=402, scale=1.0 / math.sqrt(Ci * k * k))
    sc = torch.rand(Co, generator=_g(403)) + 0.5
    bi = rnd(Co, seed=404) * 0.01
    got = _conv_p4(x, w, s, p, tile=tile, scale=sc, bias=bi)
    emu, den = _emul(x, w, s, p, frame_amax(x), scale=sc, bias=bi)
    e_emu = ((got.double() - emu).abs() / (den + 1e-30)).max().item()
    assert e_emu <= 1e-5, e_emu
    ref = ref_conv(x, w, s, p, scale=sc, bias=bi).double()
    den0 = F.conv2d(x.double().abs(), w.double().abs(), None, s, p) * sc.double().view(1, -1, 1, 1)
    e_ref = ((got.double() - ref).abs() / (den0 + 1e-30)).max().item()
    assert e_ref <= 2.0 ** -10, e_ref


@pytest.mark.parametrize("tile", [0, 24, 25, 27, 28, 29])
@pytest.mark.parametrize("stride", [1, 2])
def test_conv_p4_prologue_bound(tile, stride):
    """IR-50 res_layer: BN prologue on the input (in-bounds taps only), 3x3 conv, BN + PReLU.
    The activation scale comes from x_amax max|in_scale| + max|in_bias| (a valid bound of the
    prologue's output), so nothing overflows even with negative / large affine terms."""
    B, Ci, H, W, Co = 2, 64, 12, 14, 96
    x = rnd(B, Ci, H, W, seed=410) * 3.0
    w = rnd(Co, Ci, 3, 3, seed=411, scale=1.0 / math.sqrt(Ci * 9))
    in_s = rnd(Ci, seed=412) * 2.0
    in_b = rnd(Ci, seed=413) * 4.0
    sc = torch.rand(Co, generator=_g(414)) + 0.5
    bi = rnd(Co, seed=415)
    sl = torch.rand(Co, generator=_g(416)) * 0.3
    got = _conv_p4(x, w, stride, 1, tile=tile, in_s=in_s, in_b=in_b, act="prelu", scale=sc, bias=bi, slope=sl)
    assert torch.isfinite(got).all()
    emu, den = _emul(x, w, stride, 1, frame_amax(x), in_s=in_s, in_b=in_b, scale=sc, bias=bi, act="prelu", slope=sl)
    # PReLU slope <= 1: the pre-activation bound carries through; the prologue's fp32 fma vs the
    # emulation's mul + add may flip an fp16 rounding of an element (one 2^-12 ulp): 2e-4 margin
    e_emu = ((got.double() - emu).abs() / (den + 1e-30)).max().item()
    assert e_emu <= 2e-4, e_emu
    ref = ref_conv(x, w, stride, 1, act="prelu", scale=sc, bias=bi, slope=sl, in_s=in_s, in_b=in_b).double()
    xx = x.double() * in_s.double().view(1, -1, 1, 1) + in_b.double().view(1, -1, 1, 1)
    den0 = F.conv2d(xx.abs(), w.double().abs(), None, stride, 1) * sc.double().view(1, -1, 1, 1)
    e_ref = ((got.double() - ref).abs() / (den0 + 1e-30)).max().item()
    assert e_ref <= 2.0 ** -9, e_ref        # the bound may be up to ~2x loose: one bit of the scale


@pytest.mark.parametrize("tile", [30, 31, 32, 33, 34, 36, 37])
@pytest.mark.parametrize("B,Ci,H,W,Co", [(2, 64, 17, 19, 96), (1, 256, 33, 40, 128), (2, 32, 16, 16, 256),
                                         (2, 128, 16, 16, 64)])
def test_conv_p4_halo_bit_exact_vs_wave(B, Ci, H, W, Co, tile):
    """The haloed-tile kernel at precision 4 (one fp16 plane, B ring of the hi plane) runs the
    wave kernel's K order and per-accumulator MFMA order: bit-identical, residual + SiLU."""
    x = torch.relu(rnd(B, Ci, H, W, seed=420)) * 5.0
    w = rnd(Co, Ci, 3, 3, seed=421, scale=1.0 / math.sqrt(Ci * 9))
    sc = torch.rand(Co, generator=_g(422)) + 0.5
    bi = rnd(Co, seed=423)
    r = rnd(B, Co, H, W, seed=424)
    kw = dict(scale=sc, bias=bi, act="silu", res=r, res_mode=RES_PRE)
    a = _conv_p4(x, w, 1, 1, tile=tile, **kw)
    b = _conv_p4(x, w, 1, 1, tile=27, **kw)
    assert torch.equal(a, b)
    emu, den = _emul(x, w, 1, 1, frame_amax(x), scale=sc, bias=bi, act="silu", res=r, res_mode=RES_PRE)
    assert ((a.double() - emu).abs() / (den + 1e-30)).max().item() <= 1e-5


@pytest.mark.parametrize("tile", [0, 30, 31, 34, 36, 37])
@pytest.mark.parametrize("B,Ci,H,W,Co", [(2, 64, 17, 19, 96), (2, 128, 16, 16, 64), (1, 256, 14, 14, 256)])
def test_conv_p4_halo_prologue_bit_exact_vs_wave(B, Ci, H, W, Co, tile):
    """IR-50 res_layer on the haloed-tile kernel: the BN prologue is applied to the chunk's halo
    as it is converted to fp16 (pixels inside the frame only; the padding stays 0), with the
    activation scale from the prologue's bound -- bit-identical to the wave kernel's prologue
    (tile 27), and within the operand emulation. tile 0: the automatic choice (the halo kernel
    from 14 x 14 up)."""
    x = rnd(B, Ci, H, W, seed=440) * 3.0
    w = rnd(Co, Ci, 3, 3, seed=441, scale=1.0 / math.sqrt(Ci * 9))
    in_s = rnd(Ci, seed=442) * 2.0
    in_b = rnd(Ci, seed=443) * 4.0
    sc = torch.rand(Co, generator=_g(444)) + 0.5
    bi = rnd(Co, seed=445)
    sl = torch.rand(Co, generator=_g(446)) * 0.3
    kw = dict(in_s=in_s, in_b=in_b, act="prelu", scale=sc, bias=bi, slope=sl)
    a = _conv_p4(x, w, 1, 1, tile=tile, **kw)
    b = _conv_p4(x, w, 1, 1, tile=27, **kw)
    assert torch.equal(a, b)
    emu, den = _emul(x, w, 1, 1, frame_amax(x), in_s=in_s, in_b=in_b, scale=sc, bias=bi, act="prelu", slope=sl)
    assert ((a.double() - emu).abs() / (den + 1e-30)).max().item() <= 2e-4


def test_conv_p4_descriptor_rules():
    """precision 4 needs the fp16 plane and x_amax; no dual input, no planes format."""
    x = torch.relu(rnd(2, 64, 8, 8, seed=430)).permute(0, 2, 3, 1).contiguous().to(DEV)
    pk = pack.pack_conv("r", rnd(64, 64, 1, 1, seed=431), 1, 0, DEV)
    y = torch.empty(2, 8, 8, 64, device=DEV)
    with pytest.raises(Exception):
        ops.conv2d(x, pk, y, precision=4)                       # no x_amax
    xa = frame_amax(x.permute(0, 3, 1, 2)).to(DEV)
    with pytest.raises(Exception):
        ops.conv2d(x, pk, y, precision=4, x_amax=xa, y_planes=True)
    with pytest.raises(Exception):
        ops.conv2d(x, pk, y, precision=4, x_amax=xa, x2=x, x2_amax=xa)
    ops.conv2d(x, pk, y, precision=4, x_amax=xa)
    torch.cuda.synchronize()
    # the haloed-tile kernel's forced 16 x 16-pixel 64-column tile has no single-plane form
    pk3 = pack.pack_conv("r3", rnd(64, 64, 3, 3, seed=432), 1, 1, DEV, k_order=1)
    with pytest.raises(Exception):
        ops.conv2d(x, pk3, y, precision=4, x_amax=xa, tile=35)
    ops.conv2d(x, pk3, y, precision=4, x_amax=xa, tile=34)
    torch.cuda.synchronize()


@pytest.mark.parametrize("act", ["prelu", "gelu", "silu"])
@pytest.mark.parametrize("size,ac", [((112, 112), True), ((40, 36), True), ((64, 48), False)])
def test_upconv_frame_amax(size, ac, act):
    """prpe_upconv3x3's y_amax (ABI 8): raised to exactly max|y[n]| per frame on the LDS-DMA
    kernel (112x112 from 20x20: the AdaFace adapter) and the fused kernel (other geometries);
    the output itself is unchanged by tracking it."""
    B, Hi, Wi, Co = 3, 20, 20, 64
    z = rnd(B, Hi, Wi, 9 * Co, seed=440).to(DEV)
    z[1] *= 0.001
    sc = (torch.rand(Co, generator=_g(441)) + 0.5).to(DEV)
    bi = rnd(Co, seed=442).to(DEV)
    sl = (torch.rand(Co, generator=_g(443)) * 0.3).to(DEV)
    y = torch.empty(B, *size, Co, device=DEV)
    y0 = torch.empty(B, *size, Co, device=DEV)
    ya = torch.zeros(B, device=DEV)
    ops.upconv3x3(z, y, ac, sc, bi, sl if act == "prelu" else None, act, y_amax=ya)
    ops.upconv3x3(z, y0, ac, sc, bi, sl if act == "prelu" else None, act)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    assert torch.equal(ya.cpu(), frame_amax(y.permute(0, 3, 1, 2)))
