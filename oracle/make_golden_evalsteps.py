"""Golden fixtures made by the REFERENCE's own code in this container (import shims as in
make_golden.py; test infrastructure only, never shipped to the GPU box):

    python -B oracle/make_golden_evalsteps.py   ->  tests/golden/golden_vitpose.npz,
                                                    tests/golden/golden_flip.npz,
                                                    tests/golden/golden_facerec.npz

* golden_vitpose.npz (BASELINE config 3): transformers' ``VitPoseForPoseEstimation`` (the
  module the reference wraps, modify_models.py:383-385; site-packages modeling_vitpose.py:
  190-278) with the seed-1 weights, run directly on pixel_values U[0,1) [2,3,256,192].
* golden_flip.npz: ``PoseEstimationModule.validation_step``
  (pose_estimation/module.py:451-570) executed as written, with a stub model that returns
  given heatmaps for the original and the flipped pass; the averaged heatmaps the flip block
  (:466-484) hands to ``_get_keypoints_from_heatmaps`` are captured, plus its outputs.
* golden_facerec.npz: ``FaceRecognitionModule.validation_step``
  (face_recognition/module.py:119-157) with a stub model returning given embeddings and a
  given ``ada_face.head.kernel`` [512, C]; records val_loss / val_acc (C = 1000 classes here,
  so the fixture stays small; the kernel shape is what the code normalises, not C).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]
GOLD = os.path.join(ROOT, "tests", "golden")

from oracle import model_ref as R  # noqa: E402
from oracle import ref_shims  # noqa: E402
from oracle.fixtures import facerec_inputs, flip_inputs, vitpose_pixels  # noqa: E402
from prpe import arch, synth  # noqa: E402


def vitpose_golden(sd):
    from oracle.ref_build import vitpose_config
    from transformers import VitPoseForPoseEstimation
    vit = VitPoseForPoseEstimation(vitpose_config()).eval()
    pre = "vit_pose.vit_pose."
    vsd = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
    missing, unexpected = vit.load_state_dict(vsd, strict=False)
    assert not missing and not unexpected, (missing[:4], unexpected[:4])
    pix = vitpose_pixels()
    with torch.no_grad():
        heat = vit(pixel_values=pix).heatmaps
        mine = R.vitpose_backbone(sd, pix)
    d = float((heat - mine).abs().max())
    print(f"vitpose: oracle vs transformers max|d| = {d:.2e}")
    assert d <= 1e-4
    # inputs are regenerated bit-identically from prpe.synth by the tests; only their checksum
    # is stored beside the outputs
    np.savez_compressed(os.path.join(GOLD, "golden_vitpose.npz"), pixel_sum=np.float64(pix.double().sum()),
                        heatmaps=heat.numpy())


def _datamodule_shims():
    """The Lightning packages' __init__ import their datamodules: class-level annotations read
    albumentations attributes (A.Compose ...) and albumentations.pytorch is imported at module
    level -- inert placeholders are enough (no datamodule code runs)."""
    ref_shims.install()
    sys.modules["albumentations"].__getattr__ = lambda name: object
    if "albumentations.pytorch" not in sys.modules:
        ap = types.ModuleType("albumentations.pytorch")
        ap.ToTensorV2 = object
        sys.modules["albumentations.pytorch"] = ap


def _pose_module():
    _datamodule_shims()
    sys.modules.pop("lightning.pose_estimation.datamodule", None)   # a stub from reference_softargmax
    sys.modules.pop("lightning.pose_estimation.module", None)
    import importlib
    dm = importlib.import_module("lightning.pose_estimation.datamodule")
    assert dm.COCO_FLIP_PAIRS == R.COCO_FLIP_PAIRS
    return importlib.import_module("lightning.pose_estimation.module")


def flip_golden():
    mod = _pose_module()
    heat, heat_f = flip_inputs()
    B, K, H, W = heat.shape
    images = synth.uniform(31, "flip_images", (B, 3, 256, 192))
    calls = []

    class StubModel(torch.nn.Module):
        def set_task(self, t):
            pass

        def forward(self, x):
            calls.append(x.clone())
            from transformers.models.vitpose.modeling_vitpose import VitPoseEstimatorOutput
            return VitPoseEstimatorOutput(heatmaps=(heat if len(calls) == 1 else heat_f).clone())

    m = mod.PoseEstimationModule(StubModel())
    captured = {}
    orig = m._get_keypoints_from_heatmaps

    def grab(heatmaps, boxes=None):
        captured["avg"] = heatmaps.clone()
        captured["boxes"] = None if boxes is None else boxes.clone()
        out = orig(heatmaps, boxes=boxes)
        captured["coords"], captured["scores"] = out[0].clone(), out[1].clone()
        return out

    m._get_keypoints_from_heatmaps = grab
    boxes = synth.uniform(32, "flip_boxes", (B, 1, 4)) * 150
    boxes[..., 2:] += boxes[..., :2] + 20
    batch = {"images": images, "keypoints": torch.cat([synth.uniform(33, "flip_kp", (B, 1, K, 2)) * 100,
                                                        torch.full((B, 1, K, 1), 2.0)], -1),
             "boxes": boxes, "areas": torch.full((B, 1), 5000.0), "masks": torch.zeros(B, 1, dtype=torch.bool),
             "is_crowd": torch.zeros(B, 1, dtype=torch.bool), "image_ids": list(range(B))}
    with torch.no_grad():
        m.validation_step(batch, 0)
    assert len(calls) == 2 and torch.equal(calls[1], torch.flip(images, dims=[-1]))
    mine = R.pose_flip_average(heat, heat_f.clone(), "reference")
    assert torch.equal(mine, captured["avg"]), "oracle flip restatement != reference"
    np.savez_compressed(os.path.join(GOLD, "golden_flip.npz"), heat_sum=np.float64(heat.double().sum()),
                        heat_flipped_sum=np.float64(heat_f.double().sum()),
                        avg=captured["avg"].numpy(), boxes=captured["boxes"].numpy(),
                        coords=captured["coords"].numpy(), scores=captured["scores"].numpy())
    print("flip: avg max", float(captured["avg"].abs().max()))


def facerec_golden():
    _datamodule_shims()
    import importlib
    mod = importlib.import_module("lightning.face_recognition.module")
    emb, kernel, labels = facerec_inputs()
    B, C = emb.shape[0], kernel.shape[1]

    class StubModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.ada_face = types.SimpleNamespace(head=types.SimpleNamespace(kernel=kernel))

        def set_task(self, t):
            pass

        def forward(self, x):
            return emb.clone(), emb.norm(dim=1, keepdim=True)

    m = mod.FaceRecognitionModule(StubModel(), num_classes=C)
    m.hparams = types.SimpleNamespace(s=64.0, m=0.4, h=0.333)
    m.validation_step_outputs = []
    with torch.no_grad():
        out = m.validation_step((torch.zeros(B, 3, 112, 112), labels), 0)
    loss, acc, _, amax = R.face_recognition_eval(emb, kernel, labels, 64.0)
    assert torch.equal(loss, out["val_loss"]) and torch.equal(acc, out["val_acc"]), "oracle != reference"
    np.savez_compressed(os.path.join(GOLD, "golden_facerec.npz"), emb_sum=np.float64(emb.double().sum()),
                        kernel_sum=np.float64(kernel.double().sum()), labels=labels.numpy(), val_loss=out["val_loss"].numpy(), val_acc=out["val_acc"].numpy(),
                        argmax=amax.numpy())
    print("facerec: loss", float(out["val_loss"]), "acc", float(out["val_acc"]))


def sd_keys_golden(sd):
    """Keys and shapes of the reference CombinedModel's own state_dict() (arch.state_dict_spec
    must reproduce them; tests/test_abi_and_host.py)."""
    import json
    from oracle.ref_build import build_reference_model
    sd = dict(sd)
    sd["ada_face.head.kernel"] = torch.zeros(512, arch.ADAFACE_CLASSES)
    model = build_reference_model(sd)
    keys = {k: list(v.shape) for k, v in model.state_dict().items()}
    with open(os.path.join(GOLD, "sd_keys_ref.json"), "w") as f:
        json.dump(keys, f, indent=0)
    print("state_dict keys:", len(keys))


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    sd = synth.make_state_dict(arch.state_dict_spec())
    ref_shims.install()
    sd_keys_golden(sd)
    vitpose_golden(sd)
    flip_golden()
    facerec_golden()
    for f in ("golden_vitpose.npz", "golden_flip.npz", "golden_facerec.npz"):
        print(f, os.path.getsize(os.path.join(GOLD, f)))


if __name__ == "__main__":
    main()
