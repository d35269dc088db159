"""GPU: parity at the BASELINE batch sizes (config 4: bs=256 full model; config 2: bs=64
face-YOLO + NMS; config 3: ViTPose-B on pixel_values) and frame independence.

* Frame independence: a frame's outputs do not depend on its batch-mates (BN uses running
  statistics, the YOLO normalisation is per sample, the precision-3 activation scales are per
  frame): frames 0 / 127 / 255 of a bs=256 forward_all are BIT-IDENTICAL to the same frames
  run at bs=2. This is what makes the 8-GPU frame sharding exact.
* Parity vs the oracle (fp32 CPU restatement, pinned to the reference) on frames spread over
  the batch (0, B/3, 2B/3, B-1 -- late frames exercise the 64-bit offsets of tensors with
  more than 2^31 elements): heatmaps / embeddings / YOLO scores within 1e-3 abs, boxes within
  2e-3 x max|box|, keypoint OKS delta <= 1e-3, NMS bit-exact on our own det tensor.
* Config 3: ``model.vit_pose.vit_pose(pixel_values)`` against transformers'
  VitPoseForPoseEstimation run by the generator (tests/golden/golden_vitpose.npz).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

from oracle import model_ref as R
from oracle.fixtures import vitpose_pixels
from prpe import CombinedModel, synth
from prpe.postproc import non_max_suppression_padded

pytestmark = pytest.mark.gpu
STRIDE = [8.0, 16.0, 32.0]


def spread(B):
    return sorted({0, B // 3, (2 * B) // 3, B - 1})


@pytest.fixture(scope="module")
def model(state_dict):
    return CombinedModel(state_dict, device="cuda")


@pytest.fixture(scope="module")
def frames256():
    return synth.frames(256)


@pytest.fixture(scope="module")
def out256(model, frames256):
    o = model.forward_all(frames256.cuda(), face_stride=STRIDE)
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in o.items()}


def test_frames_independent_of_batch_bit_identical(model, frames256, out256):
    for pair in ((0, 127), (255, 1)):
        o2 = model.forward_all(frames256[list(pair)].cuda(), face_stride=STRIDE)
        for k in ("det", "emb", "norm", "heatmaps"):
            a = o2[k].cpu()
            for j, f in enumerate(pair):
                assert torch.equal(a[j], out256[k][f]), (k, f)


def test_config4_bs256_parity_on_spread_frames(state_dict, frames256, out256):
    idx = spread(256)
    with torch.no_grad():
        ref = R.forward_all(state_dict, frames256[idx], stride=STRIDE)
    e_hm = (out256["heatmaps"][idx] - ref["heatmaps"]).abs().max().item()
    e_emb = (out256["emb"][idx] - ref["emb"]).abs().max().item()
    e_cls = (out256["det"][idx, 4] - ref["det"][:, 4]).abs().max().item()
    e_box = (out256["det"][idx, :4] - ref["det"][:, :4]).abs().max().item() / ref["det"][:, :4].abs().max().item()
    c, _ = R.keypoints_from_heatmaps(out256["heatmaps"][idx])
    rc, _ = R.keypoints_from_heatmaps(ref["heatmaps"])
    oks = R.oks_delta(c, rc)
    print(f"bs256 frames {idx}: heat {e_hm:.2e} emb {e_emb:.2e} cls {e_cls:.2e} box/max {e_box:.2e} oks {oks:.1e}")
    assert e_hm <= 1e-3 and e_emb <= 1e-3 and e_cls <= 1e-3 and e_box <= 2e-3 and oks <= 1e-3
    torch.testing.assert_close(out256["norm"][idx], ref["norm"], rtol=1e-3, atol=0)


def test_config4_nms_bit_exact_on_own_det(out256):
    det = out256["det"]
    dets, cnt = non_max_suppression_padded(det.cuda())
    dets, cnt = dets.cpu(), cnt.cpu()
    for f in spread(256) + [17, 200]:
        ref = R.non_max_suppression(det[f:f + 1])[0]
        assert int(cnt[f]) == len(ref)
        assert torch.equal(dets[f, :len(ref)], ref)


def test_config2_yolo_face_bs64(model, state_dict):
    x = synth.frames(64, seed=3)
    e = model.engine
    det = e.yolo("yolo_face", e.trunk(x.cuda()), STRIDE)
    dets, cnt = non_max_suppression_padded(det)
    det, dets, cnt = det.cpu(), dets.cpu(), cnt.cpu()
    idx = spread(64)
    with torch.no_grad():
        ref = R.yolo_branch(state_dict, "yolo_face", R.resnet50_trunk(state_dict, x[idx]), STRIDE)
    assert (det[idx, 4] - ref[:, 4]).abs().max().item() <= 1e-3
    assert (det[idx, :4] - ref[:, :4]).abs().max().item() <= 2e-3 * ref[:, :4].abs().max().item()
    for j, f in enumerate(idx):
        mine = R.non_max_suppression(det[f:f + 1])[0]          # NMS bit-exact on the same tensor
        assert int(cnt[f]) == len(mine) and torch.equal(dets[f, :len(mine)], mine)
    from test_gpu_model import assert_nms_end_to_end
    # end to end, NMS runs on OUR scores, which differ from the oracle's by up to ~3e-5 (measured):
    # a pair whose suppression decision is tied to that level (IoU within rounding of 0.65, or a
    # score at the confidence threshold) could legitimately flip. Measured 1.0 on every frame in
    # rounds 3-5; a flip must be a near-tie (checked and printed), and the rate stays >= 0.98.
    assert_nms_end_to_end([dets[f, :cnt[f]] for f in idx], R.non_max_suppression(ref))


def test_config3_vitpose_from_pixels_vs_transformers_golden(model):
    with np.load(os.path.join(GOLDEN, "golden_vitpose.npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    pix = vitpose_pixels()
    assert pix.double().sum().item() == g["pixel_sum"]
    out = model.vit_pose.vit_pose(pix.cuda())              # the reference's call shape
    err = np.abs(out.heatmaps.cpu().numpy() - g["heatmaps"]).max()
    print("config 3 heatmaps vs transformers:", err)
    assert err <= 1e-3
    # NCHW pixel_values and the adapter's NHWC output take the same kernels: a contiguous NHWC
    # copy gives bit-identical heatmaps
    e = model.engine
    with e.prec("vit"):
        h2 = e.vit_backbone(pix.permute(0, 2, 3, 1).contiguous().cuda())
    assert torch.equal(h2.cpu(), out.heatmaps.cpu())


def test_config3_bs256_parity_on_spread_frames(model, state_dict):
    pix = synth.uniform(5, "pixel_values:256x256x192", (256, 3, 256, 192))
    heat = model.vitpose_from_pixels(pix.cuda()).heatmaps.cpu()
    idx = spread(256)
    with torch.no_grad():
        ref = R.vitpose_backbone(state_dict, pix[idx])
    assert (heat[idx] - ref).abs().max().item() <= 1e-3
    c, _ = R.keypoints_from_heatmaps(heat[idx])
    rc, _ = R.keypoints_from_heatmaps(ref)
    assert R.oks_delta(c, rc) <= 1e-3
    # frame independence on this path too
    h2 = model.vitpose_from_pixels(pix[[255, 0]].cuda()).heatmaps.cpu()
    assert torch.equal(h2[0], heat[255]) and torch.equal(h2[1], heat[0])


def _raw_yolo_close(det, ref):
    """Tolerances of the raw-frame YOLO. The synthetic net is ill-conditioned on raw 640x640
    frames (its BN statistics were calibrated on the adapter's output; scores saturate at 1.0):
    measured on the CPU oracle, fp32 vs fp64 moves a score by 3.1e-4 and a 2^-20 relative
    perturbation of the YOLO weights by 2.0e-3 (boxes 5e-4 of max). Any fp32 evaluation order
    lands in that band, so: every score within 4e-3 (2x the 2^-20 response), fewer than 0.1 % of
    the anchors beyond 1e-3, boxes within 2e-3 x max|box|."""
    e = (det[:, 4] - ref[:, 4]).abs()
    assert e.max().item() <= 4e-3, e.max().item()
    assert (e > 1e-3).float().mean().item() < 1e-3
    assert (det[:, :4] - ref[:, :4]).abs().max().item() <= 2e-3 * ref[:, :4].abs().max().item()


def test_config2_micro_yolo_raw_frames_vs_reference_golden(model):
    """Config-2 micro-bench variant: ``model.yolo_face.yolo(frames)`` -- YOLO
    v11n nc=1 straight on raw 640x640 frames, A = 8400 -- against the reference's own output
    (oracle/make_golden_yolo_raw.py), and the batched NMS at A = 8400 bit-exact against the
    reference's yolopt NMS on the golden's tie-free det copy."""
    with np.load(os.path.join(GOLDEN, "golden_yolo_raw.npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    x = synth.frames(2).cuda()
    model.yolo_face.yolo.head.stride = torch.tensor(STRIDE)
    try:
        det = model.yolo_face.yolo(x).cpu()
    finally:
        model.yolo_face.yolo.head.stride = torch.zeros(3)
    ref = torch.from_numpy(g["det"])
    assert det.shape == ref.shape == (2, 5, 8400)
    _raw_yolo_close(det, ref)
    dets, cnt = non_max_suppression_padded(torch.from_numpy(g["det_tiefree"]).cuda())
    assert cnt.cpu().tolist() == g["nms_count"].tolist()
    for i, n in enumerate(g["nms_count"].tolist()):
        assert torch.equal(dets[i, :n].cpu(), torch.from_numpy(g["nms_out"][i, :n]))
    # the model's own (tied) scores: bit-exact against the oracle's stable-order NMS
    dets, cnt = non_max_suppression_padded(det.cuda())
    for i, m in enumerate(R.non_max_suppression(det)):
        assert int(cnt[i]) == len(m) and torch.equal(dets[i, :len(m)].cpu(), m)


def test_config2_micro_yolo_raw_bs64_parity(model, state_dict):
    x = synth.frames(64, seed=4)
    det = model.engine.yolo_raw("yolo_face", x.cuda(), STRIDE).cpu()
    idx = spread(64)
    with torch.no_grad():
        ref = R.yolo_net(state_dict, "yolo_face", x[idx], STRIDE)
    _raw_yolo_close(det[idx], ref)
    # frame independence on this path
    d2 = model.engine.yolo_raw("yolo_face", x[[63, 0]].cuda(), STRIDE).cpu()
    assert torch.equal(d2[0], det[63]) and torch.equal(d2[1], det[0])
