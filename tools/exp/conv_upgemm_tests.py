"""Tests of the rejected upconv -> 1x1 fusion (tools/exp/conv_upgemm.patch), as they stood in
tests/test_gpu_ops.py at round 5; append to that file after applying the patch."""


@pytest.mark.parametrize("N,hi,wi,ho,wo,ac,C", [(2, 20, 20, 160, 160, True, 512), (1, 10, 12, 64, 70, True, 64),
                                              (2, 13, 9, 70, 53, False, 96), (1, 20, 20, 160, 160, False, 32)])
def test_upconv_gemm_bit_exact_vs_unfused(N, hi, wi, ho, wo, ac, C):
    """prpe_upconv_gemm (the face-YOLO adapter's .4 upconv + BN + SiLU and .7 1x1 + BN + SiLU in one
    launch) == prpe_upconv3x3 (planes output) followed by prpe_conv2d (precision 0, planes input,
    planes output) bit for bit: the same interpolation / BN / SiLU / split arithmetic and the same
    GEMM K order. Model shape (20 -> 160, 512 -> 256) and ragged ones (partial 16-pixel tiles, both
    align_corners modes, other channel counts)."""
    Co = 256
    z = rnd(N, hi, wi, 9 * C, seed=510, scale=0.5).to(DEV)
    us = (torch.rand(C, generator=_g(511)) + 0.5).to(DEV)
    ub = rnd(C, seed=512).to(DEV)
    w = rnd(Co, C, 1, 1, seed=513, scale=1.0 / math.sqrt(C))
    sc = torch.rand(Co, generator=_g(514)) + 0.5
    bi = rnd(Co, seed=515)
    pk = pack.pack_conv("ug", w, 1, 0, DEV, scale=sc, bias=bi, act="silu")
    u = torch.empty(N, ho, wo, C, device=DEV)
    ops.upconv3x3(z, u, ac, us, ub, None, "silu", y_planes=True)
    ref = torch.empty(N, ho, wo, Co, device=DEV)
    ops.conv2d(u, pk, ref, precision=0, x_planes=True, y_planes=True)
    got = torch.empty(N, ho, wo, Co, device=DEV)
    ops.upconv_gemm(z, pk, got, ac, us, ub, up_act="silu", y_planes=True)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    # and the fp32 form of the output equals the unfused fp32 GEMM
    ref32 = torch.empty(N, ho, wo, Co, device=DEV)
    ops.conv2d(u, pk, ref32, precision=0, x_planes=True)
    got32 = torch.empty(N, ho, wo, Co, device=DEV)
    ops.upconv_gemm(z, pk, got32, ac, us, ub, up_act="silu")
    torch.cuda.synchronize()
    assert torch.equal(got32, ref32)


def test_upconv_gemm_rejects():
    """A source window over 5 rows per 16-pixel tile (upsampling ratio < ~4), Co != 256 and a
    K-mismatched pack are refused (-EINVAL / ValueError), nothing is launched."""
    z = torch.zeros(1, 20, 20, 9 * 64, device=DEV)
    pk = pack.pack_conv("ug", rnd(256, 64, 1, 1, seed=520), 1, 0, DEV)
    with pytest.raises(PrpeError):
        ops.upconv_gemm(z, pk, torch.empty(1, 40, 40, 256, device=DEV), True, torch.ones(64, device=DEV),
                        torch.zeros(64, device=DEV))
    pk128 = pack.pack_conv("ug", rnd(128, 64, 1, 1, seed=521), 1, 0, DEV)
    with pytest.raises(PrpeError):
        ops.upconv_gemm(z, pk128, torch.empty(1, 160, 160, 128, device=DEV), True, torch.ones(64, device=DEV),
                        torch.zeros(64, device=DEV))
    pk32 = pack.pack_conv("ug", rnd(256, 32, 1, 1, seed=522), 1, 0, DEV)
    with pytest.raises(ValueError):
        ops.upconv_gemm(z, pk32, torch.empty(1, 160, 160, 256, device=DEV), True, torch.ones(64, device=DEV),
                        torch.zeros(64, device=DEV))
