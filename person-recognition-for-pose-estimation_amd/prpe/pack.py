"""Weight packing: reference state_dict tensors -> device-resident conv packs.

A ``ConvPack`` holds the weight of one conv / linear in the layout the implicit-GEMM
kernel streams (include/prpe.h, prpe_conv2d):
  * W[co, ci, kh, kw] -> [co][k], zero-padded to [co_pad][k_pad] (k_pad % 32 == 0,
    co_pad % 128 == 0), with k tap-major (k_order 0: k = (kh*KW + kw)*Ci + ci) or, for
    KH*KW > 1 and Ci % 32 == 0, chunk-major (k_order 1: k = ((ci/32)*KH*KW + kh*KW+kw)*32
    + ci%32, the 9 taps of one 32-channel chunk adjacent), split into three bf16 planes
    (p0 = RNE(w), p1 = RNE(w - p0), p2 = RNE(w - p0 - p1); p0+p1+p2 == w exactly);
  * the epilogue's per-channel affine: eval BatchNorm folded exactly as PyTorch's CPU
    batch_norm inference does (alpha = gamma / sqrt(var + eps), beta' = beta - mean*alpha),
    with the conv bias folded in (bias*alpha + beta');
  * optional PReLU slopes and an input-side (prologue) affine for pre-activation BN.
Packing runs once at load time (host + one upload); nothing here is on the per-frame path.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


def _rup(v: int, m: int) -> int:
    return (v + m - 1) // m * m


@dataclass
class ConvPack:
    name: str
    w_hi: torch.Tensor
    w_lo: torch.Tensor
    w_lo2: torch.Tensor
    kh: int
    kw: int
    stride: int
    pad: int
    ci: int
    co: int
    k_pad: int
    co_pad: int
    scale: torch.Tensor | None = None
    bias: torch.Tensor | None = None
    slope: torch.Tensor | None = None
    in_scale: torch.Tensor | None = None
    in_bias: torch.Tensor | None = None
    act: str = "none"
    k_order: int = 0
    f16: tuple | None = None      # (w_h16, w_l16, scale16), built on first precision-3 use
    tile: int = 0                 # kernel tile for prpe_conv2d (0 = the library's automatic choice)

    @property
    def flops_per_pixel(self) -> int:
        return 2 * self.co * self.ci * self.kh * self.kw

    def f16_planes(self):
        """Precision-3 operands (see split_f16_scaled), cached on the pack."""
        if self.f16 is None:
            w = (self.w_hi.float() + self.w_lo.float() + self.w_lo2.float()).cpu()   # exact fp32 w
            h, l, e = split_f16_scaled(w)
            sc = self.scale.cpu() if self.scale is not None else torch.ones(self.co)
            s16 = torch.ldexp(sc.float(), -e[: self.co].to(torch.int32)).float()
            dev = self.w_hi.device
            self.f16 = (h.contiguous().to(dev), l.contiguous().to(dev), s16.contiguous().to(dev))
        return self.f16


def split_bf16(w: torch.Tensor, planes: int = 3):
    """fp32 -> ``planes`` bf16 tensors (RNE splits); 3 planes reproduce fp32 exactly."""
    r = w.float()
    out = []
    for _ in range(planes):
        t = r.to(torch.bfloat16)
        out.append(t)
        r = r - t.float()
    return out


def split_f16_scaled(w2d: torch.Tensor):
    """[co, K] fp32 -> (hi, lo, e): each row scaled by 2^e[co] so its max |w| lies in
    [2^14, 2^15) (exact), then split into two fp16 planes as uint16 bits: hi = RNE(w 2^e),
    lo = RNE(w 2^e - hi); w 2^e = hi + lo to ~2^-22 relative (the lo plane may be subnormal for
    entries far below the row maximum: absolute error <= 2^-25 in scaled units). All-zero rows
    get e = 0."""
    w = w2d.float()
    m = w.abs().amax(1)
    _, ex = torch.frexp(m)                       # m = f * 2^ex, f in [0.5, 1)
    e = torch.where(m > 0, 15 - ex, torch.zeros_like(ex)).to(torch.int32)
    ws = torch.ldexp(w, e.view(-1, 1))
    hi = ws.to(torch.float16)
    lo = (ws - hi.float()).to(torch.float16)
    return hi.view(torch.int16), lo.view(torch.int16), e


def bn_affine(sd, prefix, eps, conv_bias=None):
    """(scale, shift) of an eval BatchNorm (+ preceding conv bias), fp32."""
    var = sd[prefix + ".running_var"].float()
    mean = sd[prefix + ".running_mean"].float()
    g = sd.get(prefix + ".weight")
    b = sd.get(prefix + ".bias")
    g = torch.ones_like(var) if g is None else g.float()
    b = torch.zeros_like(var) if b is None else b.float()
    alpha = g / torch.sqrt(var + eps)
    shift = b - mean * alpha
    if conv_bias is not None:
        shift = shift + conv_bias.float() * alpha
    return alpha.contiguous(), shift.contiguous()


def pack_matrix(name, w2d: torch.Tensor, kh, kw, ci, stride, pad, device, scale=None, bias=None,
                slope=None, in_scale=None, in_bias=None, act="none", k_order=0) -> ConvPack:
    """w2d: [co, K] with K in the order ``k_order`` names (see module docstring)."""
    co, K = w2d.shape
    k_pad, co_pad = _rup(K, 32), _rup(co, 128)
    wp = torch.zeros(co_pad, k_pad, dtype=torch.float32)
    wp[:co, :K] = w2d.float()
    p0, p1, p2 = split_bf16(wp, 3)
    dev = lambda t: None if t is None else t.float().contiguous().to(device)
    return ConvPack(name, p0.contiguous().to(device), p1.contiguous().to(device), p2.contiguous().to(device), kh, kw,
                    stride, pad, ci, co, k_pad, co_pad, dev(scale), dev(bias), dev(slope), dev(in_scale),
                    dev(in_bias), act, k_order)


def pack_conv(name, w: torch.Tensor, stride=1, pad=0, device="cuda", k_order="auto", **kw) -> ConvPack:
    """w: [co, ci, kh, kw] (PyTorch layout). k_order "auto" picks chunk-major whenever it
    applies (KH*KW > 1, Ci % 32 == 0); the input view must then be channel-contiguous."""
    co, ci, kh, kw_ = w.shape
    if k_order == "auto":
        k_order = 1 if kh * kw_ > 1 and ci % 32 == 0 else 0
    if k_order == 1:
        assert ci % 32 == 0, name
        w2d = w.float().reshape(co, ci // 32, 32, kh, kw_).permute(0, 1, 3, 4, 2).reshape(co, -1)
    else:
        w2d = w.float().permute(0, 2, 3, 1).reshape(co, kh * kw_ * ci)
    return pack_matrix(name, w2d, kh, kw_, ci, stride, pad, device, k_order=k_order, **kw)


def pack_upconv_taps(name, w: torch.Tensor, device="cuda") -> ConvPack:
    """3x3 conv weight [co, ci, 3, 3] -> 1x1 pack with 9*co outputs (channel = tap*co + co'):
    stage 1 of the exact upsample/conv rewrite (prpe_upconv3x3)."""
    co, ci, kh, kw_ = w.shape
    assert kh == 3 and kw_ == 3
    w2d = w.float().permute(2, 3, 0, 1).reshape(9 * co, ci)   # [(tap, co), ci]
    return pack_matrix(name, w2d, 1, 1, ci, 1, 0, device)
