"""CPU: host logic of the eval-step mirrors (no device calls)."""
import torch

from oracle import model_ref as R
from prpe.evalsteps import COCO_FLIP_PAIRS, flip_partner


def test_flip_partner_is_an_involution():
    p = flip_partner(17)
    assert p[0] == -1
    for a, b in COCO_FLIP_PAIRS:
        assert p[a] == b and p[b] == a


def test_reference_flip_pairs_reverse_the_batch():
    """module.py:482-483 ``flipped[:, pair] = flipped[:, pair].flip(0)``: for paired channels
    the batch order is reversed (not the pair's channels swapped) -- the device kernel's
    mode 0 reproduces exactly this index map."""
    B, K, H, W = 3, 17, 2, 5
    h = torch.zeros(B, K, H, W)
    f = torch.arange(B * K * H * W, dtype=torch.float32).view(B, K, H, W)
    out = R.pose_flip_average(h, f.clone(), "reference") * 2
    part = flip_partner(K)
    for b in range(B):
        for k in range(K):
            b2 = B - 1 - b if part[k] >= 0 else b
            assert torch.equal(out[b, k], torch.flip(f[b2, k], dims=[-1]))
    swap = R.pose_flip_average(h, f.clone(), "swap") * 2
    for k in range(K):
        k2 = part[k] if part[k] >= 0 else k
        assert torch.equal(swap[:, k], torch.flip(f[:, k2], dims=[-1]))


def _golden_detmetrics():
    import os
    import numpy as np
    return dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_detmetrics.npz")))


def test_detection_metrics_oracle_matches_reference_golden():
    """oracle.DetectionMetricsRef == the reference's DetectionMetrics (module_v2.py:13-127) as
    driven by validation_step, on the fixtures it produced (oracle/make_golden_detmetrics.py):
    counters, (score, is_tp, iou) records in order, and every compute() value."""
    g = _golden_detmetrics()
    m = R.DetectionMetricsRef()
    for b in range(2):
        dets, counts = torch.from_numpy(g[f"dets{b}"]), torch.from_numpy(g[f"counts{b}"])
        preds = [dets[i, :int(counts[i])] for i in range(dets.shape[0])]
        m.update_batch(preds, torch.from_numpy(g[f"gt{b}"]), torch.from_numpy(g[f"gtidx{b}"]))
    assert [m.tp, m.fp, m.gt, len(m.records)] == g["counters"].tolist()
    rec = torch.tensor([[s, float(t), v] for s, t, v in m.records], dtype=torch.float64)
    assert torch.equal(rec, torch.from_numpy(g["records"]))
    out = m.compute()
    got = [out[k] for k in ("precision", "recall", "f1", "mAP50", "mAP75", "mAP")]
    assert got == g["metrics"].tolist()
    # the fixture covers the reference's edge cases
    assert any(r[2] == 0.5 for r in m.records)                       # IoU exactly 0.5: not a TP
    scores = [r[0] for r in m.records]
    assert len(set(scores)) < len(scores)                            # tied scores


def test_detection_eval_loss_oracle_matches_reference_golden():
    """oracle.detection_eval_loss_ref == the reference's FaceDetectionModule.compute_loss on
    its own fixtures (oracle/make_golden_detmetrics.py): the batch loss and each image's
    terms, incl. images without ground truth, without kept predictions, without positives."""
    import math
    import os
    import numpy as np
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_detloss.npz")))
    det = torch.from_numpy(g["det"])
    gt, gidx = torch.from_numpy(g["gt"]), torch.from_numpy(g["gtidx"])
    loss, per = R.detection_eval_loss_ref(det[:, :4], det[:, 4:5], gt, torch.zeros(len(gt), dtype=torch.int64), gidx)
    assert abs(loss.item() - float(g["loss"])) <= 1e-6
    for b in range(det.shape[0]):
        exp = g["per_image"][b]
        if math.isnan(exp[0]):
            assert b not in per
            continue
        for v, e in zip(per[b], exp):
            assert (math.isnan(v) and math.isnan(e)) or abs(v - e) <= 1e-6, (b, per[b], exp)
