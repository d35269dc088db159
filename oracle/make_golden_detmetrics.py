"""Golden fixtures for the device DetectionMetrics, made by the
reference's OWN classes in this container (import shims as in make_golden.py; test
infrastructure only, never shipped to the GPU box):

    python -B oracle/make_golden_detmetrics.py   ->  tests/golden/golden_detmetrics.npz,
                                                    tests/golden/golden_detloss.npz

Inputs: two synthetic batches of padded NMS outputs [B, 300, 6] + counts and ground-truth
boxes with batch indices, with the edge cases the reference code distinguishes: images with
no prediction, images with no ground truth, tied scores (stable sort order), a prediction at
IoU exactly 0.5 (not a TP, kept at the 0.5 threshold), and predictions far from any box.
Outputs: the reference's counters, its (score, is_tp, iou) records and compute() dict,
after FaceDetectionModule.validation_step's own update loop (module_v2.py:480-499).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ref_shims  # noqa: E402


def make_batch(seed, B=6, cap=300):
    g = torch.Generator().manual_seed(seed)
    dets = torch.zeros(B, cap, 6)
    counts = torch.zeros(B, dtype=torch.int32)
    gts, gidx = [], []
    for i in range(B):
        ng = [3, 0, 5, 2, 4, 1][i % 6]
        n = [40, 25, 0, 300, 60, 7][i % 6]
        c = torch.rand(ng, 2, generator=g) * 500
        wh = torch.rand(ng, 2, generator=g) * 100 + 10
        gb = torch.cat([c, c + wh], 1)
        gts.append(gb)
        gidx += [i] * ng
        if n == 0:
            continue
        # predictions: jittered copies of the boxes + random boxes; scores with ties
        k = torch.randint(0, max(ng, 1), (n,), generator=g)
        base = gb[k] if ng else torch.rand(n, 4, generator=g) * 500
        jit = (torch.rand(n, 4, generator=g) - 0.5) * 40
        pb = base + jit
        pb[:, 2:] = torch.maximum(pb[:, 2:], pb[:, :2] + 1)
        far = torch.rand(n, generator=g) < 0.2
        pb[far] += 2000
        sc = torch.round(torch.rand(n, generator=g) * 20) / 20 + 0.001        # many ties
        order = torch.argsort(sc, descending=True, stable=True)               # NMS output order
        pb, sc = pb[order], sc[order]
        if ng and n > 1:
            # IoU exactly 0.5: same y-extent, x-extent covering half the box width
            b = gb[0].clone()
            pb[1] = torch.tensor([b[0], b[1], b[0] + (b[2] - b[0]) / 2, b[3]])
        dets[i, :n, :4] = pb
        dets[i, :n, 4] = sc
        counts[i] = n
    return dets, counts, torch.cat(gts, 0), torch.tensor(gidx, dtype=torch.int64)


def loss_inputs(seed=21, B=6, N=525):
    """Eval head output [B, 5, N] (boxes taken as xyxy, as compute_loss does; scores in (0, 1))
    with per-image cases: positives and negatives, no ground truth, nothing above 0.01, kept
    predictions but no positive, many positives with a single negative."""
    g = torch.Generator().manual_seed(seed)
    det = torch.zeros(B, 5, N)
    gts, gidx = [], []
    for i in range(B):
        ng = [3, 0, 2, 4, 1, 2][i]
        c = torch.rand(ng, 2, generator=g) * 400
        gb = torch.cat([c, c + torch.rand(ng, 2, generator=g) * 80 + 20], 1)
        gts.append(gb)
        gidx += [i] * ng
        k = torch.randint(0, max(ng, 1), (N,), generator=g)
        base = gb[k] if ng else torch.rand(N, 4, generator=g) * 400
        pb = base + (torch.rand(N, 4, generator=g) - 0.5) * 30
        sc = torch.rand(N, generator=g)
        if i == 2:
            sc = sc * 0.009                       # nothing above the 0.01 filter
        if i == 3:
            pb = pb + 1000                        # kept, but no positive
        if i == 5:
            # eight kept positives and a single kept negative (a one-element background mean)
            sc = torch.where(torch.arange(N) < 9, sc * 0.5 + 0.5, sc * 0.005)
            pb[:8] = gb[k[:8]] + (torch.rand(8, 4, generator=g) - 0.5) * 2
            pb[8] = pb[8] + 1000
        det[i, :4] = pb.t()
        det[i, 4] = sc
    return det, torch.cat(gts, 0), torch.tensor(gidx, dtype=torch.int64)


def golden_loss(module_cls):
    class _M(torch.nn.Module):
        def set_task(self, t):
            pass
    mod = module_cls(_M())
    det, gt, gidx = loss_inputs()
    boxes, scores = mod.process_yolo_output(det, is_training=False)
    import contextlib, io
    with contextlib.redirect_stdout(io.StringIO()):
        loss, d = mod.compute_loss(boxes, scores, {"boxes": gt, "labels": torch.zeros(len(gt), dtype=torch.int64),
                                                   "batch_idx": gidx})
    per = np.full((det.shape[0], 4), np.nan)
    for b in range(det.shape[0]):
        if f"box_loss_{b}" in d:
            per[b] = [d[f"box_loss_{b}"] + d[f"cls_loss_{b}"] + 0.5 * d[f"bg_loss_{b}"], d[f"box_loss_{b}"],
                      d[f"cls_loss_{b}"], d[f"bg_loss_{b}"]]
        elif f"bg_loss_{b}" in d:
            per[b] = [d[f"bg_loss_{b}"], np.nan, np.nan, d[f"bg_loss_{b}"]]
    path = os.path.join(ROOT, "tests", "golden", "golden_detloss.npz")
    np.savez_compressed(path, det=det.numpy(), gt=gt.numpy(), gtidx=gidx.numpy(), loss=np.float64(loss.item()),
                        per_image=per)
    print(path, loss.item())


def main():
    ref_shims.install()
    from lightning.face_detection.module_v2 import DetectionMetrics, FaceDetectionModule  # the reference
    golden_loss(FaceDetectionModule)

    m = DetectionMetrics()
    out = {}
    for bi, seed in enumerate((11, 12)):
        dets, counts, gt, gidx = make_batch(seed)
        out[f"dets{bi}"], out[f"counts{bi}"] = dets.numpy(), counts.numpy()
        out[f"gt{bi}"], out[f"gtidx{bi}"] = gt.numpy(), gidx.numpy()
        preds = [dets[i, :int(counts[i])] for i in range(dets.shape[0])]
        for i, pred in enumerate(preds):                       # module_v2.py:480-499
            if len(pred) == 0:
                continue
            mask = gidx == i
            gb, gc = gt[mask], torch.zeros(int(mask.sum()), dtype=torch.int64)
            if len(gb) == 0:
                continue
            m.update(pred[:, :4], pred[:, 4], pred[:, 5].long(), gb, gc)
    res = m.compute()
    out["counters"] = np.array([m.total_tp, m.total_fp, m.total_gt, len(m.ap_scores)], dtype=np.int64)
    out["records"] = np.array([[s, float(t), v] for s, t, v in m.ap_scores], dtype=np.float64)
    out["metrics"] = np.array([res[k] for k in ("precision", "recall", "f1", "mAP50", "mAP75", "mAP")])
    path = os.path.join(ROOT, "tests", "golden", "golden_detmetrics.npz")
    np.savez_compressed(path, **out)
    print(path, {k: round(float(v), 6) for k, v in res.items()}, out["counters"].tolist())


if __name__ == "__main__":
    main()
