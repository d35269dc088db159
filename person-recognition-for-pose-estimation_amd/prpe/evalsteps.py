"""Device halves of the reference eval steps that wrap the model.

* ``pose_flip_test``  — PoseEstimationModule.validation_step's flip test
  (training/lightning/pose_estimation/module.py:466-484): heatmaps of the frames and of the
  W-mirrored frames (the mirror is a negative-stride read in the stem's layout kernel, no
  flipped copy), flipped back and averaged by one kernel (prpe_flip_average). ``mode``:
  "reference" reproduces ``flipped[:, pair] = flipped[:, pair].flip(0)`` literally (that
  reverses the BATCH order of the paired channels); "swap" exchanges the pair's channels.
* ``FaceRecognitionEval`` — FaceRecognitionModule.validation_step's head
  (training/lightning/face_recognition/module.py:133-145): F.normalize of the [512, classes]
  head kernel (rows, dim=1) once per kernel, then per batch F.normalize(embeddings), the
  [B,512] x [512,classes] cosine GEMM with the scale s folded into the epilogue (prpe_conv2d,
  fp32-faithful 3-plane mode), and cross-entropy + argmax + accuracy on device
  (prpe_ce_argmax).
* ``DetectionMetricsDevice`` — the detection validation step's DetectionMetrics
  (training/lightning/face_detection/module_v2.py:13-127, driven by validation_step :458-499):
  per batch one launch matches the padded NMS output against the ground truth and appends
  (score, best IoU) records on device (prpe_det_metrics_update); compute() at epoch end
  (prpe_det_metrics_compute) returns the reference's dict.
* ``detection_eval_loss`` — the same step's compute_loss (module_v2.py:178-303) on the eval
  head output: one block per image (confidence filter, IoU matching, the pairwise CIoU mean,
  cross-entropy, background BCE), no per-image host sync (prpe_det_eval_loss).
"""
from __future__ import annotations

import torch

from . import ops
from .pack import pack_matrix

F_NORMALIZE_EPS = 1e-12          # torch.nn.functional.normalize default eps
COCO_FLIP_PAIRS = [(1, 2), (3, 4), (5, 6), (7, 8), (9, 10), (11, 12), (13, 14), (15, 16)]  # datamodule.py:25-34


def flip_partner(k: int = 17, pairs=COCO_FLIP_PAIRS) -> list[int]:
    part = [-1] * k
    for a, b in pairs:
        part[a], part[b] = b, a
    return part


@torch.no_grad()
def pose_flip_test(model, images, mode: str = "reference"):
    """Averaged flip-test heatmaps [B,17,64,48] for ``images`` [B,3,H,W] (module.py:466-484)."""
    if mode not in ("reference", "swap"):
        raise ValueError(f"unknown flip mode {mode!r}")
    x = model._check_input(images)
    model._sync_weights()                         # repack if a weight changed in place
    e = model.engine
    heat = e.vitpose(e.trunk(x))
    heat_f = e.vitpose(e.trunk(x, flip_w=True))
    return ops.flip_average(heat, heat_f, flip_partner(heat.shape[1]), 0 if mode == "reference" else 1)


class FaceRecognitionEval:
    """(loss, acc) of the face-recognition eval step, on device."""

    def __init__(self, model, s: float = 64.0, precision: int = 2):
        kernel = model.ada_face.head.kernel
        if kernel is None:
            raise ValueError("model.ada_face.head.kernel is not set (load a state_dict that has it)")
        self.model = model
        self.s = float(s)
        self.precision = precision
        self.set_kernel(kernel)

    def set_kernel(self, kernel):
        """Normalise + pack the [512, classes] head kernel. An in-place change of ``kernel``
        (the model's ``ada_face.head.kernel`` parameter) is detected by its version counter at
        the next call and repacked, as ``CombinedModel`` does for its weights."""
        self._kernel, self._kernel_version = kernel, kernel._version
        k = kernel.to(self.model.device, torch.float32).contiguous()
        d, ncls = k.shape
        kn = torch.empty_like(k)
        ops.l2norm(k, kn, torch.empty(d, device=k.device), F_NORMALIZE_EPS)   # F.normalize(kernel), dim=1
        self.classes = ncls
        self.pack = pack_matrix("ada_face.head:logits", kn.t().cpu(), 1, 1, d, 1, 0, self.model.device,
                                scale=torch.full((ncls,), self.s))

    def logits(self, embeddings):
        if self._kernel._version != self._kernel_version:
            self.set_kernel(self._kernel)
        B, d = embeddings.shape
        e = embeddings.contiguous().float()
        en = torch.empty_like(e)
        ops.l2norm(e, en, torch.empty(B, device=e.device), F_NORMALIZE_EPS)   # F.normalize(embeddings)
        out = torch.empty(B, 1, 1, self.classes, device=e.device)
        ops.conv2d(en.view(B, 1, 1, d), self.pack, out, precision=self.precision)
        return out.view(B, self.classes)

    @torch.no_grad()
    def __call__(self, images=None, labels=None, embeddings=None):
        """Returns (loss, acc, argmax) as device tensors; pass ``embeddings`` to skip the model."""
        if embeddings is None:
            self.model.set_task("face_recognition")
            embeddings, _ = self.model(images)
        out = self.logits(embeddings)
        loss, amax, summary = ops.ce_argmax(out, labels)
        if labels is None:
            return None, None, amax
        return summary[0], summary[1], amax


class DetectionMetricsDevice:
    """DetectionMetrics with its state on the device (same update/compute semantics)."""

    THRESHOLDS = torch.linspace(0.5, 0.95, 10).tolist()     # module_v2.py:92
    KEYS = ("precision", "recall", "f1", "mAP50", "mAP75", "mAP")

    def __init__(self, device="cuda", capacity: int = 1 << 20):
        self.counters = torch.zeros(4, dtype=torch.int64, device=device)   # tp, fp, gt, records
        self.records = torch.empty(capacity, 2, dtype=torch.float32, device=device)

    def reset(self):
        self.counters.zero_()

    def update_batch(self, dets, counts, gt_boxes, gt_batch):
        """dets [B, max_det, 6] + counts [B] (postproc.non_max_suppression_padded); gt_boxes [G, 4]
        xyxy with gt_batch [G] = the reference's targets['boxes'] / targets['batch_idx']."""
        ops.det_metrics_update(dets, counts, gt_boxes, gt_batch, self.counters, self.records)

    def compute(self) -> dict:
        n = int(self.counters[3].item())          # one host read per epoch
        if n > self.records.shape[0]:
            raise RuntimeError(f"DetectionMetricsDevice: {n} records exceed the capacity {self.records.shape[0]}")
        out = ops.det_metrics_compute(self.counters, self.records, n, self.THRESHOLDS).tolist()
        return dict(zip(self.KEYS, out))


@torch.no_grad()
def detection_eval_loss(det, gt_boxes, gt_batch, gt_labels=None):
    """(avg_loss [1], per_image [B, 4] = (loss_b, box, cls, bg)) for the eval-mode detection
    output ``det`` [B, 4+nc, N] (FaceDetectionModule.process_yolo_output's eval split:
    boxes det[:, :4], scores det[:, 4:]) against targets boxes / batch_idx / labels."""
    return ops.det_eval_loss(det[:, :4], det[:, 4:], gt_boxes, gt_batch, gt_labels)
