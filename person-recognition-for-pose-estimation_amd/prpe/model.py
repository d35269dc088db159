"""Drop-in for the reference ``CombinedModel`` (training/modify_models.py:462-494) on MI355X.

Same surface the eval steps touch:
  * ``set_task(name)`` with the reference's supported list and ValueError message;
  * ``model(images)`` routes the trunk features to one branch and returns the reference's
    per-task types: detection -> Tensor [B, 4+1, 525]; pose -> object with ``.heatmaps``
    [B,17,64,48]; face_recognition -> (embeddings [B,512], norms [B,1]);
  * ``state_dict()/load_state_dict()`` with the reference's 2130 keys;
  * parameters stay live: an in-place change through ``parameters()`` / ``state_dict()`` (an
    optimizer step in ``pl.Trainer.fit``, round_robin_trainer.py:258-262, before validation)
    is seen at the next call and the engine repacks (``_sync_weights``), so a forward never
    computes with stale packed weights;
  * ``model.yolo_face.yolo.head.stride`` / ``yolo_person...`` (a fresh ``Head`` after
    ``modify_yolo`` has stride zeros, nn.py:238 -> eval boxes are 0; honoured as given);
  * ``model.ada_face.head.kernel`` for the face-recognition eval logits;
  * the branches as ``nn.Module`` trees with the reference's parameter names
    (``model.vit_pose.adapter.parameters()``, ``model.yolo_face.parameters()`` ..., prpe.modules)
    and ``model.vit_pose.vit_pose(pixel_values)`` -> ``.heatmaps`` (BASELINE config 3).
Plus ``forward_all(x)``: trunk once, then face-YOLO + AdaFace + ViTPose (BASELINE config 4).

Eval-only: the reference's training outputs/backward are out of scope.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass
from types import SimpleNamespace

import torch

from . import arch, ops
from .engine import Engine
from .modules import branch_trees


@dataclass
class PoseOutput:
    """Stands in for transformers' VitPoseEstimatorOutput (the callers read ``.heatmaps``)."""
    heatmaps: torch.Tensor
    loss: torch.Tensor | None = None


class CombinedModel:
    SUPPORTED_TASKS = ["face_detection", "person_detection", "pose_estimation", "face_recognition"]

    def __init__(self, state_dict: dict | None = None, device="cuda", precision="auto"):
        self.current_task = "person_detection"
        self.device = torch.device(device)
        self.training = False
        self.precision = precision
        self._sd = {}
        self.yolo_face = SimpleNamespace(yolo=SimpleNamespace(head=SimpleNamespace(stride=torch.zeros(3))))
        self.yolo_person = SimpleNamespace(yolo=SimpleNamespace(head=SimpleNamespace(stride=torch.zeros(3))))
        self.ada_face = SimpleNamespace(head=SimpleNamespace(kernel=None))
        self.vit_pose = None
        self.engine = None
        if state_dict is not None:
            self.load_state_dict(state_dict)

    # ------------------------------------------------------------------ nn.Module-like API
    def load_state_dict(self, state_dict, strict: bool = True):
        keys = {k for k, _, _ in arch.state_dict_spec()}
        missing = [k for k in keys if k not in state_dict and k != "ada_face.head.kernel"]
        unexpected = [k for k in state_dict if k not in keys]
        if strict and (missing or unexpected):
            raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
        strides = {b: getattr(self, b).yolo.head.stride for b in ("yolo_face", "yolo_person")}
        self._sd = {k: v.detach().cpu() for k, v in state_dict.items()}
        trees = branch_trees(self._sd, self)
        for b, t in trees.items():
            setattr(self, b, t)
        for b, st in strides.items():          # a reload keeps the stride the caller set
            getattr(self, b).yolo.head.stride = st
        self.engine = Engine(self._sd, self.device, self.precision)
        self._mark_packed()
        return SimpleNamespace(missing_keys=missing, unexpected_keys=unexpected)

    # ------------------------------------------------------------------ weight freshness
    # The HIP engine computes from packed device copies of ``_sd`` (split planes, folded BN).
    # Every tensor the caller can reach -- the branch trees' parameters / buffers, the trunk's
    # ``parameters()``, ``state_dict()`` values -- shares storage AND autograd's version counter
    # with its ``_sd`` entry (nn.Parameter(t) / t.detach() alias t), so any in-place write through
    # them (``p.add_``, ``p.copy_``, an optimizer step) bumps that entry's ``_version``. The
    # versions are recorded when the engine packs; every entry point compares them first and
    # repacks on a change. (``p.data.<op>_`` bypasses the version counter by PyTorch's design:
    # call ``refresh_weights()`` after such writes.)
    def _mark_packed(self):
        self._packed = [(t, t._version) for t in self._sd.values()]

    def weights_stale(self) -> bool:
        """True if a state_dict tensor changed in place since the engine packed it."""
        return any(t._version != v for t, v in getattr(self, "_packed", ()))

    def refresh_weights(self):
        """Repack every weight from the (possibly edited) state_dict tensors."""
        self.engine = Engine(self._sd, self.device, self.precision)
        self._mark_packed()

    def _sync_weights(self):
        if self.engine is None:
            raise RuntimeError("no weights loaded: call load_state_dict first")
        if self.weights_stale():
            self.refresh_weights()

    def state_dict(self):
        return dict(self._sd)

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("prpe runs on MI355X (HIP) only; no CPU path")
        if device != self.device:
            self.device = device
            if self._sd:
                self.load_state_dict(self._sd, strict=False)
        return self

    def float(self):
        return self

    # parameters of the branches (the trunk's are in the state_dict under ``backbone.``)
    def parameters(self, recurse: bool = True):
        trunk = (torch.nn.Parameter(v) for k, v in self._sd.items()
                 if k.startswith("backbone.") and torch.is_floating_point(v) and "running_" not in k)
        return itertools.chain(trunk, *(getattr(self, b).parameters() for b in
                                        ("yolo_face", "yolo_person", "ada_face", "vit_pose")))

    def eval(self):
        self.training = False
        return self

    def train(self, mode: bool = True):
        if mode:
            raise NotImplementedError("training-mode outputs/backward are out of scope (eval hot path only)")
        return self.eval()

    def set_task(self, task_name):
        if task_name not in self.SUPPORTED_TASKS:
            raise ValueError(f"Task {task_name} not supported. Available tasks: {', '.join(self.SUPPORTED_TASKS)}")
        self.current_task = task_name

    # ------------------------------------------------------------------ forward
    def _check_input(self, x):
        if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
                and x.shape[1] == 3):
            raise ValueError("expected float32 CUDA(HIP) frames [B,3,H,W]")
        return x

    @torch.no_grad()
    def forward(self, x):
        x = self._check_input(x)
        self._sync_weights()
        e = self.engine
        feat = e.trunk(x)
        t = self.current_task
        if t == "pose_estimation":
            return PoseOutput(heatmaps=e.vitpose(feat))
        if t == "person_detection":
            return e.yolo("yolo_person", feat, self._stride(self.yolo_person))
        if t == "face_detection":
            return e.yolo("yolo_face", feat, self._stride(self.yolo_face))
        return e.adaface(feat)

    __call__ = forward

    @torch.no_grad()
    def vitpose_from_pixels(self, pixel_values):
        """``VitPoseForPoseEstimation(pixel_values)`` (site-packages modeling_vitpose.py:190-278),
        as the reference calls it at modify_models.py:383-385: pixel_values [B,3,256,192] ->
        PoseOutput(heatmaps [B,17,64,48]). BASELINE config 3."""
        x = pixel_values
        if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
                and tuple(x.shape[1:]) == (3,) + tuple(arch.VIT_IMG)):
            raise ValueError(f"expected float32 CUDA(HIP) pixel_values [B,3,{arch.VIT_IMG[0]},{arch.VIT_IMG[1]}]")
        self._sync_weights()
        e = self.engine
        with e.prec("vit"):
            return PoseOutput(heatmaps=e.vit_backbone(ops.nhwc(x)))

    @torch.no_grad()
    def yolo_from_frames(self, branch, x):
        """``model.<branch>.yolo(frames)``: yolopt ``YOLO.forward`` eval (nn.py:294-297) on
        [B,3,H,W] frames (H, W multiples of 32) -> [B, 5, A] with the branch head's stride
        (A = 8400 at 640x640; SURVEY.md §8d config-2 micro-bench variant)."""
        x = self._check_input(x)
        if x.shape[2] % 32 or x.shape[3] % 32:
            raise ValueError("YOLO input H and W must be multiples of 32 (the P5 stride)")
        self._sync_weights()
        return self.engine.yolo_raw(branch, x, self._stride(getattr(self, branch)))

    @torch.no_grad()
    def forward_all(self, x, face_stride=None, concurrent=True):
        """Trunk once -> face-YOLO det, AdaFace (emb, norm), ViTPose heatmaps.

        ``concurrent``: the three heads only share the trunk features, so they are enqueued on
        three HIP streams (forked from / joined back into the caller's stream by events). The
        heads' HBM-bound kernels (upsample-conv, pointwise) then co-reside on the CUs with the
        other heads' MFMA-bound convs, and one kernel's tail wave no longer idles the chip.
        Same kernels, same arithmetic: results are bit-identical to the sequential order."""
        x = self._check_input(x)
        self._sync_weights()
        e = self.engine
        feat = e.trunk(x)
        stride = face_stride if face_stride is not None else self._stride(self.yolo_face)
        heads = (lambda: e.yolo("yolo_face", feat, stride), lambda: e.adaface(feat), lambda: e.vitpose(feat))
        if not concurrent:
            det, (emb, norm), heat = (h() for h in heads)
            return {"det": det, "emb": emb, "norm": norm, "heatmaps": heat}
        main = torch.cuda.current_stream(feat.device)
        if getattr(self, "_head_streams", None) is None or self._head_streams[0].device != feat.device:
            self._head_streams = [torch.cuda.Stream(feat.device) for _ in heads]
        fork = main.record_event()
        outs = []
        for s, h in zip(self._head_streams, heads):
            s.wait_event(fork)
            feat.record_stream(s)            # feat is freed on `main`; keep it alive for `s`
            with torch.cuda.stream(s):
                outs.append(h())
        for s in self._head_streams:
            main.wait_stream(s)
        det, (emb, norm), heat = outs
        for t in (det, emb, norm, heat):
            t.record_stream(main)            # allocated on a head stream, consumed on `main`
        return {"det": det, "emb": emb, "norm": norm, "heatmaps": heat}

    @staticmethod
    def _stride(branch):
        s = branch.yolo.head.stride
        return [float(v) for v in (s.tolist() if isinstance(s, torch.Tensor) else s)]
