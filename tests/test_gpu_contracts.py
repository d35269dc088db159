"""GPU: the C-ABI contract and the geometries that were not covered before round 3.

* The split-K path (IR-50 output layer, conv_splitk.hip) takes its partial-sum workspace from
  the caller (prpe_conv2d_workspace_bytes, SURVEY.md §8b: "caller allocates every buffer ...
  safe to call concurrently on different streams"): two streams running it at once give
  results bit-identical to sequential runs.
* The dual-input conv3 + downsample GEMM at the model's layer1.0 geometry at bs=256 (M = 6.55 M
  rows, x2 the full-resolution block input as a stride-1 view, precision 3) against fp64 on
  sampled rows, including the last rows of the last frame (64-bit offsets past 2^31 elements).
* precision 3 outside the trunk (an Engine policy of 3 everywhere): forward_all and
  vitpose_from_pixels run (per-component max|y| slot pools) and stay within the model
  tolerances of the reference's golden outputs.
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN
from prpe import CombinedModel, ops, pack, synth
from test_gpu_ops import DEV, _g, rnd

pytestmark = pytest.mark.gpu


def _ir50_output_pack(seed):
    Ci, H, Co = 512, 7, 512
    w = rnd(Co, Ci, H, H, seed=seed, scale=1.0 / (Ci * H * H) ** 0.5)
    sc = torch.rand(Co, generator=_g(seed + 1)) + 0.5
    bi = rnd(Co, seed=seed + 2)
    ins = torch.rand(Ci, generator=_g(seed + 3)) + 0.5
    inb = rnd(Ci, seed=seed + 4)
    return w, pack.pack_conv("ir50.output", w, 1, 0, DEV, scale=sc, bias=bi, in_scale=ins, in_bias=inb, k_order=0)


def test_splitk_workspace_concurrent_streams_bit_identical():
    _, pk = _ir50_output_pack(300)
    xs = [torch.rand(256, 7, 7, 512, generator=torch.Generator(DEV).manual_seed(s), device=DEV) for s in (1, 2)]
    seq = []
    for x in xs:
        y = torch.empty(256, 1, 1, 512, device=DEV)
        ops.conv2d(x, pk, y)
        seq.append(y)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in xs]
    for _rep in range(3):
        outs = [torch.empty(256, 1, 1, 512, device=DEV) for _ in xs]
        ev = torch.cuda.current_stream().record_event()
        for s, x, y in zip(streams, xs, outs):
            s.wait_event(ev)
            with torch.cuda.stream(s):           # each call's workspace comes from its own stream
                for _ in range(4):
                    ops.conv2d(x, pk, y)
        torch.cuda.synchronize()
        for a, b in zip(outs, seq):
            assert torch.equal(a, b)
    # (the split-K numerics vs fp64: test_gpu_ops.test_conv_splitk_linear)


def test_dual_input_layer1_geometry_bs256_precision3():
    """layer1.0 conv3 + downsample (o: conv2 output [256,160,160,64], x2: the maxpool output,
    stride 1) as one precision-3 GEMM, 64 + 64 -> 256, ReLU: fp64 on 4,160 sampled rows."""
    B, H, W, C, Co = 256, 160, 160, 64, 256
    gen = torch.Generator(DEV).manual_seed(7)
    o = torch.relu(torch.randn(B, H, W, C, generator=gen, device=DEV))
    xb = torch.relu(torch.randn(B, H, W, C, generator=gen, device=DEV)) * 3.0
    w = rnd(Co, 2 * C, seed=301, scale=0.12)
    bias = rnd(Co, seed=302)
    pk = pack.pack_matrix("dual", w, 1, 1, 2 * C, 1, 0, DEV, bias=bias, act="relu")
    oa = o.abs().flatten(1).amax(1).contiguous()
    xa = xb.abs().flatten(1).amax(1).contiguous()
    y = torch.empty(B, H, W, Co, device=DEV)
    ya = torch.zeros(B, device=DEV)
    ops.conv2d(o, pk, y, precision=3, x_amax=oa, x2=xb[:, ::1, ::1, :], x2_amax=xa, y_amax=ya)
    torch.cuda.synchronize()
    M = B * H * W
    g = torch.Generator().manual_seed(8)
    rows = torch.cat([torch.randint(0, M, (4000,), generator=g), torch.arange(M - 128, M), torch.arange(32)])
    a = torch.cat([o.view(M, C)[rows.to(DEV)], xb.view(M, C)[rows.to(DEV)]], 1).cpu().double()
    ref = torch.relu(a @ w.double().T + bias.double())
    got = y.view(M, Co)[rows.to(DEV)].cpu().double()
    den = a.abs() @ w.double().abs().T + 1e-30
    err = ((got - ref).abs() / den).max().item()
    assert err < 2 ** -20, err
    # per-frame max|y| slots of the frames touched by the sampled rows (first, last)
    for f in (0, B - 1):
        assert float(ya[f]) == float(y[f].abs().max())


@pytest.fixture(scope="module")
def model_p3(state_dict):
    return CombinedModel(state_dict, device="cuda", precision=3)


def test_precision3_everywhere_forward_all(model_p3, golden_model):
    frames = synth.frames(2).cuda()
    for concurrent in (False, True):
        o = model_p3.forward_all(frames, face_stride=[8.0, 16.0, 32.0], concurrent=concurrent)
        assert np.abs(o["heatmaps"].cpu().numpy() - golden_model["heatmaps"]).max() <= 1e-3
        assert np.abs(o["emb"].cpu().numpy() - golden_model["emb"]).max() <= 1e-3
        np.testing.assert_allclose(o["det"].cpu().numpy()[:, 4], golden_model["det_face_s8"][:, 4], atol=1e-3)
    # slot pools are per component and reused across forwards: a second forward is identical
    o2 = model_p3.forward_all(frames, face_stride=[8.0, 16.0, 32.0])
    for k in ("det", "emb", "heatmaps"):
        assert torch.equal(o2[k], o[k]), k


def test_precision3_vitpose_from_pixels(model_p3):
    import os
    from oracle.fixtures import vitpose_pixels
    with np.load(os.path.join(GOLDEN, "golden_vitpose.npz"), allow_pickle=False) as z:
        ref = z["heatmaps"]
    out = model_p3.vitpose_from_pixels(vitpose_pixels().cuda())
    assert np.abs(out.heatmaps.cpu().numpy() - ref).max() <= 1e-3
