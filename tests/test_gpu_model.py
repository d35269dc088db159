"""GPU: the full HIP hot path (prpe.CombinedModel) against the reference's golden outputs on
the same seeded frames/weights (bs=2, 640x640) and against the oracle.

Tolerances (north_star): heatmaps and face embeddings within 1e-3 abs of the fp32 CPU
reference; norms within 1e-3 relative; detection tensor within 1e-3 abs on cls scores
and 2e-3 x max|box| on pixel box coordinates (stride-8..32 scaled; measured 1.4 px on
~930 px); keypoint OKS delta <= 1e-3; NMS on our own det output is bit-exact
vs the oracle NMS of the same tensor, and the end-to-end detection match vs the reference's
NMS on the reference's det tensor is 1.0 (measured; tests/test_gpu_batch.py covers bs=64/256).
"""
import numpy as np
import pytest
import torch

from oracle import model_ref as R
from prpe import CombinedModel, synth
from prpe.postproc import keypoints_from_heatmaps, non_max_suppression

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(state_dict):
    return CombinedModel(state_dict, device="cuda")


@pytest.fixture(scope="module")
def frames():
    return synth.frames(2).cuda()


def test_face_detection_zero_stride_quirk(model, frames, golden_model):
    model.set_task("face_detection")
    det = model(frames).cpu().numpy()
    ref = golden_model["det_face_s0"]
    assert det.shape == ref.shape == (2, 5, 525)
    assert np.all(det[:, :4] == 0)                       # Head.stride zeros -> boxes 0
    np.testing.assert_allclose(det[:, 4], ref[:, 4], rtol=0, atol=1e-3)


def test_person_detection_branch(model, frames, golden_model):
    model.set_task("person_detection")
    det = model(frames).cpu().numpy()
    np.testing.assert_allclose(det[:, 4], golden_model["det_person_s0"][:, 4], rtol=0, atol=1e-3)


def test_face_detection_with_strides(model, frames, golden_model):
    model.set_task("face_detection")
    model.yolo_face.yolo.head.stride = torch.tensor([8.0, 16.0, 32.0])
    try:
        det = model(frames).cpu().numpy()
    finally:
        model.yolo_face.yolo.head.stride = torch.zeros(3)
    ref = golden_model["det_face_s8"]
    np.testing.assert_allclose(det[:, 4], ref[:, 4], rtol=0, atol=1e-3)
    # pixel boxes (DFL expectation x stride 8..32) amplify logit rounding: an all-fp32-faithful
    # run (precision=2 everywhere) differs by 0.48 px, "auto" by ~1.5 px on ~750-930 px
    # coordinates (tools/precision_sweep.py); tolerance 2e-3 x max coordinate
    np.testing.assert_allclose(det[:, :4], ref[:, :4], rtol=0, atol=2e-3 * np.abs(ref[:, :4]).max())


def test_pose_heatmaps_and_keypoints(model, frames, golden_model):
    model.set_task("pose_estimation")
    out = model(frames)
    hm = out.heatmaps
    ref = golden_model["heatmaps"]
    err = np.abs(hm.cpu().numpy() - ref).max()
    assert err <= 1e-3, err
    c, s = keypoints_from_heatmaps(hm)
    cr, sr = R.keypoints_from_heatmaps(torch.from_numpy(ref))
    assert R.oks_delta(c.cpu(), cr) <= 1e-3
    np.testing.assert_allclose(s.cpu().numpy(), sr.numpy(), rtol=1e-3)


def test_face_recognition_embeddings(model, frames, golden_model):
    model.set_task("face_recognition")
    emb, norm = model(frames)
    e = np.abs(emb.cpu().numpy() - golden_model["emb"]).max()
    assert e <= 1e-3, e
    np.testing.assert_allclose(norm.cpu().numpy(), golden_model["norm"], rtol=1e-3)
    np.testing.assert_allclose(np.linalg.norm(emb.cpu().numpy(), axis=1), 1.0, rtol=1e-5)


def test_forward_all_matches_per_task(model, frames, golden_model):
    o = model.forward_all(frames, face_stride=[8.0, 16.0, 32.0])
    assert np.abs(o["heatmaps"].cpu().numpy() - golden_model["heatmaps"]).max() <= 1e-3
    assert np.abs(o["emb"].cpu().numpy() - golden_model["emb"]).max() <= 1e-3
    np.testing.assert_allclose(o["det"].cpu().numpy()[:, 4], golden_model["det_face_s8"][:, 4], atol=1e-3)


def test_forward_all_concurrent_heads_bit_identical(model, frames):
    # the three heads on their own streams run the same kernels as the sequential order
    a = model.forward_all(frames, face_stride=[8.0, 16.0, 32.0], concurrent=True)
    b = model.forward_all(frames, face_stride=[8.0, 16.0, 32.0], concurrent=False)
    for k in ("det", "emb", "norm", "heatmaps"):
        assert torch.equal(a[k], b[k]), k


def test_nms_on_model_output_bit_exact_vs_oracle(model, frames, golden_model):
    o = model.forward_all(frames, face_stride=[8.0, 16.0, 32.0])
    det = o["det"]
    ours = non_max_suppression(det)
    theirs = R.non_max_suppression(det.cpu())
    for a, b in zip(ours, theirs):
        np.testing.assert_array_equal(a.cpu().numpy(), b.numpy())
    # end-to-end agreement with the reference's NMS on the reference's own det tensor: NMS is
    # discontinuous in its inputs, so report the fraction of reference detections that have a
    # same-class match (IoU >= 0.9, |score diff| < 1e-3) among ours (hard parts)
    ref = R.non_max_suppression(torch.from_numpy(golden_model["det_face_s8"]))
    assert_nms_end_to_end([a.cpu() for a in ours], ref)


def _iou(a, b):
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:4], b[None, :, 2:4])
    inter = (rb - lt).clamp(min=0).prod(-1)
    area = lambda t: (t[:, 2] - t[:, 0]) * (t[:, 3] - t[:, 1])
    return inter / (area(a)[:, None] + area(b)[None, :] - inter)


def _matched(a, b):
    """[len(a)] bool: row i of a has a same-class row in b with IoU >= 0.9 and |score diff| < 1e-3."""
    if len(a) == 0 or len(b) == 0:
        return torch.zeros(len(a), dtype=torch.bool)
    ok = (_iou(a, b) >= 0.9) & ((a[:, None, 4] - b[None, :, 4]).abs() < 1e-3) & (a[:, None, 5] == b[None, :, 5])
    return ok.any(1)


def nms_match_rate(ours, ref):
    if len(ref) == 0:
        return 1.0 if len(ours) == 0 else 0.0
    return float(_matched(ref, ours).float().mean())


def unexplained_nms_flips(ours, ref, iou_thr=0.65, conf_thr=0.001, eps=2e-3):
    """Rows of either list without a match in the other that are NOT explained by a near-tie of
    the greedy NMS (end to end, NMS runs on scores that differ from the oracle's by
    ~3e-5, so a decision tied to that level may legitimately flip): a row is explained when its
    score is within eps of the confidence threshold, or some row of either list overlaps it with
    an IoU within eps of the IoU threshold (the suppression test IoU > thr can go either way)."""
    out = []
    both = torch.cat([ours, ref]) if len(ours) and len(ref) else (ours if len(ours) else ref)
    for a, b in ((ours, ref), (ref, ours)):
        miss = ~_matched(a, b)
        for r in a[miss]:
            near_conf = abs(float(r[4]) - conf_thr) < eps
            iou = _iou(r[None], both)[0]
            near_iou = bool(((iou - iou_thr).abs() < eps).any())
            if not (near_conf or near_iou):
                out.append(r.tolist())
    return out


def assert_nms_end_to_end(ours_list, ref_list, floor=0.98):
    """End-to-end NMS agreement: every frame's match rate >= floor, and every mismatch a near-tie
    (printed, so a flip is looked at rather than absorbed by the floor)."""
    rates = [nms_match_rate(a, b) for a, b in zip(ours_list, ref_list)]
    print("end-to-end NMS detection match rate vs reference:", rates)
    for f, (a, b) in enumerate(zip(ours_list, ref_list)):
        if rates[f] < 1.0 or len(a) != len(b):
            bad = unexplained_nms_flips(a, b)
            print(f"frame {f}: match rate {rates[f]:.4f}, {len(a)} vs {len(b)} rows, unexplained flips: {bad}")
            assert not bad, (f, bad)
    assert min(rates) >= floor, rates


def test_inplace_weight_edit_is_never_stale(state_dict, frames):
    """an in-place edit through ``parameters()`` (what an optimizer
    step in pl.Trainer.fit does before validation, round_robin_trainer.py:258-262) must reach
    the next forward. The edited model is checked against the oracle on its own state_dict."""
    sd = {k: v.clone() for k, v in state_dict.items()}     # the session fixture stays unedited
    m = CombinedModel(sd, device="cuda")
    m.set_task("pose_estimation")
    h0 = m(frames).heatmaps.cpu()
    assert not m.weights_stale()
    named = dict(m.vit_pose.adapter.named_parameters())
    with torch.no_grad():
        named["7.weight"].mul_(1.5)                        # the dominant conv (modify_models.py:366)
        named["8.bias"].add_(0.25)                         # its BatchNorm (folded at pack time)
    assert m.weights_stale()
    h1 = m(frames).heatmaps.cpu()
    assert not m.weights_stale()
    ref = R.combined_forward(m.state_dict(), frames.cpu(), "pose_estimation")
    assert float((h1 - h0).abs().max()) > 1e-2               # the edit changes the output ...
    assert float((h1 - ref).abs().max()) <= 1e-3             # ... and the engine follows it
    # the trunk through CombinedModel.parameters() and an edit through state_dict() values
    p = next(iter(m.parameters()))
    with torch.no_grad():
        p.mul_(0.75)
        m.state_dict()["vit_pose.adapter.11.bias"].add_(0.1)
    assert m.weights_stale()
    h2 = m(frames).heatmaps.cpu()
    ref2 = R.combined_forward(m.state_dict(), frames.cpu(), "pose_estimation")
    assert float((h2 - ref2).abs().max()) <= 1e-3


def test_vit_patch_embedding_view_matches_plain_conv(model, frames, monkeypatch):
    """Round 6: the ViTPose patch embedding runs as a 16x1/16 conv over the overlapping view of the
    zero-bordered NHWC4 crops (Engine.vit_pix4, written in place by the adapter's last conv, or by
    copy_pad from caller pixel_values). Same function as the 16x16/16 pad-2 conv on the 3-channel
    crops (PRPE_VIT_PATCH_VIEW=0): different K order, so within fp32 rounding, not bit-identical;
    both through the model (adapter path) and from pixel values (config 3)."""
    from prpe import engine as E
    model.set_task("pose_estimation")
    h_view = model(frames).heatmaps.cpu()
    pix = synth.uniform(7, "pixel_values:2x256x192", (2, 3, 256, 192)).cuda()
    p_view = model.vitpose_from_pixels(pix).heatmaps.cpu()
    monkeypatch.setattr(E, "PATCH_VIEW", False)
    h_plain = model(frames).heatmaps.cpu()
    p_plain = model.vitpose_from_pixels(pix).heatmaps.cpu()
    assert float((h_view - h_plain).abs().max()) <= 5e-5
    assert float((p_view - p_plain).abs().max()) <= 5e-5
