"""Build the *reference* CombinedModel (training/modify_models.py:462-534) from the
reference's own classes, with locally generated component checkpoints instead of the
network downloads (CONTAINER-ONLY; used to pin the oracle and to make golden vectors).

The reference constructors load component checkpoints with ``torch.load``:
  * ``modify_yolo`` (modify_models.py:156-180) loads ``{'model': yolo_v11_n(80)}``
  * ``CustomAdaFace`` (modify_models.py:225-286) loads ``{'state_dict': IR-50}``
Those files are written here, by this script, into a temp dir (our own pickles).
ViTPose uses ``VitPoseForPoseEstimation(VitPoseConfig(...))`` with the
vitpose-base-simple shape instead of ``from_pretrained``.
Afterwards every parameter/buffer is overwritten from a state_dict we pass in.
"""
from __future__ import annotations

import contextlib
import io
import os
import tempfile

import torch

from . import ref_shims


def vitpose_config():
    from transformers import VitPoseConfig, VitPoseBackboneConfig
    bb = VitPoseBackboneConfig(out_indices=[12], image_size=[256, 192], patch_size=[16, 16],
                               hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                               mlp_ratio=4, hidden_act="gelu", layer_norm_eps=1e-12, qkv_bias=True)
    return VitPoseConfig(backbone_config=bb, num_labels=17, use_simple_decoder=True, scale_factor=4)


def build_reference_model(state_dict=None):
    """Return the reference ``CombinedModel`` in eval mode (stdout of its prints muted)."""
    ref_shims.install()
    with contextlib.redirect_stdout(io.StringIO()):
        import modify_models as mm
        from yolopt.nets.nn import yolo_v11_n
        import net_adaface
        from transformers import VitPoseForPoseEstimation

        torch.manual_seed(0)
        with tempfile.TemporaryDirectory() as td:
            ypath = os.path.join(td, "yolo11n.pt")
            torch.save({"model": yolo_v11_n(80)}, ypath)
            apath = os.path.join(td, "adaface_ir50_ms1mv2.ckpt")
            torch.save({"state_dict": net_adaface.build_model("ir_50").state_dict()}, apath)
            yolo_person = mm.modify_yolo(ypath)
            yolo_face = mm.modify_yolo(ypath)
            ada = mm.CustomAdaFace(apath, mm.Config())
        vit = mm.CustomVitPose(VitPoseForPoseEstimation(vitpose_config()))
        backbone = mm.MultiTaskResNetFeatureExtractor(ref_shims._resnet50())
        model = mm.CombinedModel(backbone, yolo_face, yolo_person, ada, vit)
    model.eval()
    if state_dict is not None:
        missing, unexpected = model.load_state_dict(state_dict, strict=False)
        if missing or unexpected:
            raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    return model


def reference_nms():
    """``yolopt.util.non_max_suppression`` with its wall-clock cut-off disabled
    (util.py:133-134,166-167 read ``time()``; a frozen clock makes the cut-off never
    fire, so the golden output does not depend on this machine's speed)."""
    ref_shims.install()
    import yolopt.util as yu
    yu.time = lambda: 0.0
    return yu.non_max_suppression


def reference_softargmax():
    """Unbound ``PoseEstimationModule._get_keypoints_from_heatmaps`` (module.py:237-296)."""
    ref_shims.install()
    import importlib
    import sys
    import types
    # the pose module does `from .datamodule import COCO_*`; provide just those names so
    # the heavy datamodule (cv2/albumentations) is not needed.
    if "lightning.pose_estimation.datamodule" not in sys.modules:
        dm = types.ModuleType("lightning.pose_estimation.datamodule")
        dm.COCO_KEYPOINTS = []
        dm.COCO_FLIP_PAIRS = []
        dm.COCO_SIGMAS = []
        dm.PoseEstimationDataModule = object
        sys.modules["lightning.pose_estimation.datamodule"] = dm
    mod = importlib.import_module("lightning.pose_estimation.module")
    fn = mod.PoseEstimationModule._get_keypoints_from_heatmaps
    return lambda heatmaps, boxes=None: fn(None, heatmaps, boxes)
