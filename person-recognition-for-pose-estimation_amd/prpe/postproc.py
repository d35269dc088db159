"""Drop-ins for the reference's eval-step post-processing, on device.

* ``non_max_suppression`` — yolopt.util.non_max_suppression (training/yolopt/util.py:123-169):
  same signature and return type (list of [n_i, 6] tensors). Runs the batched HIP kernel
  (prpe_nms); building the Python list needs the per-image counts on the host (one sync,
  as the reference's per-image loop already implies). ``non_max_suppression_padded``
  returns the padded device result and counts with no host sync.
  Deviation: the wall-clock cut-off (util.py:133-134,166-167) is not reproduced (it makes
  the reference's output depend on machine speed).
* ``keypoints_from_heatmaps`` — PoseEstimationModule._get_keypoints_from_heatmaps
  (training/lightning/pose_estimation/module.py:237-296) -> (coords [B,K,2], scores [B,K]).
"""
from __future__ import annotations

import torch

from . import ops


def non_max_suppression_padded(outputs: torch.Tensor, confidence_threshold=0.001, iou_threshold=0.65,
                               max_det=300, max_nms=30000):
    """outputs [B, 4+nc, N] -> (dets [B, max_det, 6], counts [B] int32), no host sync."""
    return ops.nms(outputs.float(), 0, confidence_threshold, iou_threshold, max_nms, max_det)


def non_max_suppression(outputs: torch.Tensor, confidence_threshold=0.001, iou_threshold=0.65):
    out, cnt = non_max_suppression_padded(outputs, confidence_threshold, iou_threshold)
    counts = cnt.tolist()
    if any(c < 0 for c in counts):
        raise RuntimeError("prpe_nms: candidate overflow")
    return [out[i, :c] for i, c in enumerate(counts)]


def keypoints_from_heatmaps(heatmaps: torch.Tensor, boxes: torch.Tensor | None = None):
    return ops.softargmax(heatmaps.float(), boxes)
