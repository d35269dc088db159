"""Golden fixtures for the device DetectionMetrics, made by the
reference's OWN class in this container (import shims as in make_golden.py; test
infrastructure only, never shipped to the GPU box):

    python -B oracle/make_golden_detmetrics.py   ->  tests/golden/golden_detmetrics.npz

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


def main():
    ref_shims.install()
    from lightning.face_detection.module_v2 import DetectionMetrics  # the reference class

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
