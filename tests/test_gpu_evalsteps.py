"""GPU: the eval-step kernels around the model against the
REFERENCE's own validation steps (tests/golden/golden_flip.npz, golden_facerec.npz:
oracle/make_golden_evalsteps.py executed PoseEstimationModule.validation_step, module.py:
451-570, and FaceRecognitionModule.validation_step, face_recognition/module.py:119-157, in the
build container with stub models; inputs rebuilt by oracle/fixtures.py) and against the
oracle's restatements (oracle/model_ref.py pose_flip_average / face_recognition_eval, which the
generator checked bit-exact against those runs).

Tolerances: flip average bit-exact on the same heatmaps (same (a + b) * 0.5 in fp32); the
end-to-end flip test within the heatmap bar (1e-3 abs); cross-entropy within 1e-5 relative
(double-accumulated logsumexp vs torch's fp32), argmax exact except where the top-2 logits
of a row are closer than 1e-4 (fp32 GEMM rounding can swap a near-tie).
"""
import pytest
import torch

import os

import numpy as np

from oracle import model_ref as R
from oracle.fixtures import facerec_inputs, flip_inputs
from prpe import CombinedModel, ops, synth
from prpe.evalsteps import FaceRecognitionEval, flip_partner, pose_flip_test

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["reference", "swap"])
def test_flip_average_bit_exact(mode):
    g = torch.Generator().manual_seed(5)
    heat = torch.rand(3, 17, 64, 48, generator=g)
    heat_f = torch.rand(3, 17, 64, 48, generator=g)
    got = ops.flip_average(heat.cuda(), heat_f.cuda(), flip_partner(17), 0 if mode == "reference" else 1)
    ref = R.pose_flip_average(heat, heat_f.clone(), mode)
    assert torch.equal(got.cpu(), ref)


def _golden(name):
    with np.load(os.path.join(os.path.dirname(__file__), "golden", name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_flip_average_vs_reference_validation_step():
    """prpe_flip_average (mode 0) == the averaged heatmaps the reference's flip block handed to
    _get_keypoints_from_heatmaps, bit for bit; prpe_softargmax on them == its coords/scores."""
    g = _golden("golden_flip.npz")
    heat, heat_f = flip_inputs()
    assert heat.double().sum().item() == g["heat_sum"] and heat_f.double().sum().item() == g["heat_flipped_sum"]
    got = ops.flip_average(heat.cuda(), heat_f.cuda(), flip_partner(17), 0)
    assert np.array_equal(got.cpu().numpy(), g["avg"])
    c, s = ops.softargmax(got, boxes=torch.from_numpy(g["boxes"]).cuda())
    np.testing.assert_allclose(c.cpu().numpy(), g["coords"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(s.cpu().numpy(), g["scores"], rtol=1e-6, atol=1e-7)


def test_face_recognition_eval_vs_reference_validation_step(model):
    """FaceRecognitionEval on the reference validation step's inputs: val_loss / val_acc."""
    g = _golden("golden_facerec.npz")
    emb, kernel, labels = facerec_inputs()
    assert emb.double().sum().item() == g["emb_sum"] and kernel.double().sum().item() == g["kernel_sum"]
    model.ada_face.head.kernel = kernel.cuda()
    fr = FaceRecognitionEval(model, s=64.0)
    loss, acc, amax = fr(embeddings=emb.cuda(), labels=labels.cuda())
    assert abs(loss.item() - float(g["val_loss"])) <= 1e-5 * max(1.0, abs(float(g["val_loss"])))
    assert acc.item() == float(g["val_acc"])
    assert np.array_equal(amax.cpu().numpy().astype(np.int64), g["argmax"])


def test_flip_average_rejects_bad_args():
    from prpe._lib import PrpeError
    h = torch.rand(1, 17, 4, 4, device="cuda")
    with pytest.raises(PrpeError):
        ops.flip_average(h, h, flip_partner(17), mode=2)
    with pytest.raises(PrpeError):
        ops.flip_average(h, h, [40] * 17, mode=0)


@pytest.fixture(scope="module")
def model(state_dict):
    return CombinedModel(state_dict, device="cuda")


def test_pose_flip_test_matches_explicit_flip(model):
    """the negative-stride mirrored read == running the model on torch.flip(frames)"""
    x = synth.frames(2).cuda()
    got = pose_flip_test(model, x, "reference")
    model.set_task("pose_estimation")
    h = model(x).heatmaps
    hf = model(torch.flip(x, dims=[-1]).contiguous()).heatmaps
    ref = R.pose_flip_average(h.cpu(), hf.cpu(), "reference")
    assert torch.equal(got.cpu(), ref)


def test_pose_flip_test_vs_oracle(model, state_dict):
    x = synth.frames(2)
    got = pose_flip_test(model, x.cuda(), "reference").cpu()
    with torch.no_grad():
        h = R.vitpose_branch(state_dict, R.resnet50_trunk(state_dict, x))
        hf = R.vitpose_branch(state_dict, R.resnet50_trunk(state_dict, torch.flip(x, dims=[-1])))
    ref = R.pose_flip_average(h, hf, "reference")
    assert (got - ref).abs().max().item() <= 1e-3


def test_ce_argmax_vs_torch():
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(37, 1000, generator=g) * 20
    logits[3, 10] = logits[3, 500] = 1e4           # tie: first index wins
    labels = torch.randint(0, 1000, (37,), generator=g)
    loss, amax, summary = ops.ce_argmax(logits.cuda(), labels.cuda())
    ref_rows = torch.nn.functional.cross_entropy(logits.double(), labels, reduction="none")
    torch.testing.assert_close(loss.cpu().double(), ref_rows, rtol=1e-6, atol=1e-5)
    assert torch.equal(amax.cpu().long(), logits.max(1)[1])
    assert amax[3].item() == 10
    s = summary.cpu()
    assert abs(s[0].item() - ref_rows.mean().item()) <= 1e-5 * max(1.0, ref_rows.mean().item())
    assert s[1].item() == (logits.max(1)[1] == labels).float().mean().item()


def test_face_recognition_eval_vs_oracle(model):
    g = torch.Generator().manual_seed(11)
    emb = torch.nn.functional.normalize(torch.randn(64, 512, generator=g))
    labels = torch.randint(0, 85742, (64,), generator=g)
    kernel = synth.head_kernel()
    model.ada_face.head.kernel = kernel.cuda()
    fr = FaceRecognitionEval(model, s=64.0)
    loss, acc, amax = fr(embeddings=emb.cuda(), labels=labels.cuda())
    rl, racc, rout, ramax = R.face_recognition_eval(emb, kernel, labels, 64.0)
    out = fr.logits(emb.cuda()).cpu()
    torch.testing.assert_close(out, rout, rtol=0, atol=2e-4)      # |logit| <= 64
    top2 = rout.topk(2, dim=1).values
    near_tie = (top2[:, 0] - top2[:, 1]) < 1e-4
    mism = amax.cpu().long() != ramax
    assert not torch.any(mism & ~near_tie)
    assert abs(loss.item() - rl.item()) <= 1e-4 * max(1.0, abs(rl.item()))
    if not torch.any(near_tie):
        assert acc.item() == racc.item()


def _golden_detmetrics():
    import os
    import numpy as np
    return dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_detmetrics.npz")))


def test_detection_metrics_device_vs_reference_golden():
    """Device DetectionMetrics on the reference's own fixtures: counters and records exact
    (IoUs bit-exact), precision/recall/f1 exact, APs to fp32 summation order (1e-6)."""
    from prpe.evalsteps import DetectionMetricsDevice
    g = _golden_detmetrics()
    m = DetectionMetricsDevice("cuda", capacity=4096)
    for b in range(2):
        m.update_batch(torch.from_numpy(g[f"dets{b}"]).cuda(), torch.from_numpy(g[f"counts{b}"]).cuda(),
                       torch.from_numpy(g[f"gt{b}"]).cuda(), torch.from_numpy(g[f"gtidx{b}"]).cuda())
    torch.cuda.synchronize()
    assert m.counters.cpu().tolist() == g["counters"].tolist()
    n = int(g["counters"][3])
    rec = m.records[:n].cpu().double()
    ref = torch.from_numpy(g["records"])
    assert torch.equal(rec[:, 0], ref[:, 0]) and torch.equal(rec[:, 1], ref[:, 2])
    out = m.compute()
    keys = ("precision", "recall", "f1", "mAP50", "mAP75", "mAP")
    for k, v in zip(keys, g["metrics"].tolist()):
        if k in ("precision", "recall", "f1"):
            assert out[k] == v, k
        else:
            assert abs(out[k] - v) <= 1e-6 * max(1.0, abs(v)), (k, out[k], v)
    m.reset()
    assert all(v == 0.0 for v in m.compute().values())


def test_detection_metrics_device_large_vs_oracle():
    """Many batches (records span several 2048-record scan tiles), the oracle as reference."""
    from oracle import model_ref as R
    from prpe.evalsteps import DetectionMetricsDevice
    gen = torch.Generator().manual_seed(5)
    m = DetectionMetricsDevice("cuda", capacity=1 << 16)
    ref = R.DetectionMetricsRef()
    for _ in range(6):
        B, cap = 16, 300
        dets = torch.zeros(B, cap, 6)
        counts = torch.randint(0, cap + 1, (B,), generator=gen, dtype=torch.int32)
        ng = torch.randint(0, 6, (B,), generator=gen)
        gt = torch.cat([torch.cat([c := torch.rand(int(k), 2, generator=gen) * 400,
                                   c + torch.rand(int(k), 2, generator=gen) * 80 + 5], 1) for k in ng])
        gidx = torch.repeat_interleave(torch.arange(B), ng)
        for i in range(B):
            n = int(counts[i])
            sc = torch.sort(torch.round(torch.rand(n, generator=gen) * 50) / 50, descending=True, stable=True)[0]
            c = torch.rand(n, 2, generator=gen) * 400
            dets[i, :n, :2], dets[i, :n, 2:4] = c, c + torch.rand(n, 2, generator=gen) * 80 + 5
            dets[i, :n, 4] = sc
        m.update_batch(dets.cuda(), counts.cuda(), gt.cuda(), gidx.cuda())
        ref.update_batch([dets[i, :int(counts[i])] for i in range(B)], gt, gidx)
    assert m.counters.cpu().tolist() == [ref.tp, ref.fp, ref.gt, len(ref.records)]
    assert len(ref.records) > 3 * 2048
    out, exp = m.compute(), ref.compute()
    for k in exp:
        assert abs(out[k] - exp[k]) <= 1e-5 * max(1.0, abs(exp[k])), (k, out[k], exp[k])


def test_detection_eval_loss_device_vs_reference_golden():
    """Device compute_loss on the reference's own fixtures: batch loss and per-image terms
    (fp32 libm and reduction order: 2e-5)."""
    import math
    import os
    import numpy as np
    from prpe.evalsteps import detection_eval_loss
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_detloss.npz")))
    det = torch.from_numpy(g["det"]).cuda()
    loss, per = detection_eval_loss(det, torch.from_numpy(g["gt"]).cuda(), torch.from_numpy(g["gtidx"]).cuda())
    torch.cuda.synchronize()
    assert abs(loss.item() - float(g["loss"])) <= 2e-5
    per = per.cpu().double().numpy()
    for b in range(det.shape[0]):
        exp = g["per_image"][b]
        if math.isnan(exp[0]):
            assert per[b, 0] == 0.0          # no term for this image
            continue
        for v, e in zip(per[b], exp):
            assert (math.isnan(v) and math.isnan(e)) or abs(v - e) <= 2e-5, (b, per[b], exp)


def test_detection_eval_loss_all_positive_is_nan_like_the_reference():
    """Every kept prediction positive: the reference's background mean is over an empty tensor
    (NaN), so its loss is NaN; the device kernel reproduces it."""
    from prpe.evalsteps import detection_eval_loss
    gt = torch.tensor([[10., 10., 50., 60.]])
    det = torch.zeros(1, 5, 4)
    det[0, :4] = torch.tensor([[10., 10., 50., 60.]] * 2 + [[0., 0., 1., 1.]] * 2).t()
    det[0, 4] = torch.tensor([0.9, 0.8, 0.001, 0.002])
    loss, per = detection_eval_loss(det.cuda(), gt.cuda(), torch.zeros(1, dtype=torch.int64).cuda())
    ref_loss, _ = R.detection_eval_loss_ref(det[:, :4], det[:, 4:5], gt, torch.zeros(1, dtype=torch.int64),
                                            torch.zeros(1, dtype=torch.int64))
    assert torch.isnan(ref_loss) and torch.isnan(loss.cpu()).all()
