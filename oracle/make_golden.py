"""Generate tests/golden/*.npz from the REFERENCE itself (container only).

Imports /root/reference with the shims of oracle/ref_shims.py (no command was denied;
SURVEY.md §8c), builds the reference ``CombinedModel`` with the seed-1 synthetic
state_dict (prpe.synth + calibrated BN stats), and records:

  * golden_model.npz   - eval outputs of ``CombinedModel.forward`` per task on 2 frames
                         (seed 0): det with the reference's default zero stride and with
                         stride [8,16,32], heatmaps, emb, norm; checksums of inputs/weights.
  * golden_nms.npz     - ``yolopt.util.non_max_suppression`` on (a) the det output
                         ([B,5,525], correct layout), (b) the eval-step layout [B,525,5]
                         (module_v2.py:474-477), (c) a clustered-box stress case.
  * golden_softargmax.npz - ``PoseEstimationModule._get_keypoints_from_heatmaps`` on the
                         model heatmaps and on peaky synthetic heatmaps with boxes.

Run: ``PYTHONDONTWRITEBYTECODE=1 python -m oracle.make_golden``
It also asserts that the oracle restatement (oracle/model_ref.py) matches the reference.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd"))
GOLD = os.path.join(ROOT, "tests", "golden")

from prpe import arch, synth  # noqa: E402
from oracle import model_ref as R  # noqa: E402
from oracle.ref_build import build_reference_model, reference_nms, reference_softargmax  # noqa: E402

import contextlib  # noqa: E402
import io  # noqa: E402


def _pack_dets(dets, cap=300):
    """list of [n_i, 6] -> padded [B, cap, 6] + counts [B]."""
    b = len(dets)
    out = np.zeros((b, cap, 6), np.float32)
    cnt = np.zeros((b,), np.int32)
    for i, d in enumerate(dets):
        n = d.shape[0]
        out[i, :n] = d.numpy()
        cnt[i] = n
    return out, cnt


def _rowsort(t):
    """Sort rows lexicographically (for multiset comparison)."""
    t = t.clone()
    for c in reversed(range(t.shape[1])):
        t = t[torch.sort(t[:, c], stable=True)[1]]
    return t


def nms_stress_input(b=4, n=2000, seed=7):
    """Clustered boxes in cx,cy,w,h with many overlaps."""
    u = synth.uniform(seed, "nms_stress", (b, 6, n))
    cx = (u[:, 0] * 8).floor() * 80 + 40 + u[:, 1] * 20
    cy = (u[:, 2] * 8).floor() * 80 + 40 + u[:, 3] * 20
    w = 20 + u[:, 4] * 60
    h = 20 + u[:, 5] * 60
    score = synth.uniform(seed, "nms_stress_score", (b, n))  # tie-free (tie order is unspecified upstream)
    return torch.stack([cx, cy, w, h, score], 1).float()


def peaky_heatmaps(b=3, k=17, h=64, w=48, seed=9):
    u = synth.uniform(seed, "peaky", (b, k, h, w), -1.0, 1.0)
    yy, xx = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32),
                            indexing="ij")
    c = synth.uniform(seed, "peaky_c", (b, k, 2))
    cy = c[..., 0:1, None] * (h - 1)
    cx = c[..., 1:2, None] * (w - 1)
    g = torch.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / 8.0) * 12.0
    return (u + g).float()


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    os.makedirs(GOLD, exist_ok=True)
    sd = synth.make_state_dict(arch.state_dict_spec())
    sd["ada_face.head.kernel"] = torch.zeros(512, arch.ADAFACE_CLASSES)
    model = build_reference_model(sd)
    x = synth.frames(2)
    res = {}
    with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
        for task in arch.TASKS:
            model.set_task(task)
            out = model(x)
            if task == "pose_estimation":
                res["heatmaps"] = out.heatmaps
            elif task == "face_recognition":
                res["emb"], res["norm"] = out
            else:
                res[f"det_{task.split('_')[0]}_s0"] = out
        model.yolo_face.yolo.head.stride = torch.tensor([8.0, 16.0, 32.0])
        model.set_task("face_detection")
        res["det_face_s8"] = model(x)
        res["feat_chsum"] = model.backbone(x).sum(dim=(2, 3))

    # oracle vs reference
    with torch.no_grad():
        o = R.forward_all(sd, x)
        o0 = R.yolo_branch(sd, "yolo_face", o["feat"], (0.0, 0.0, 0.0))
    checks = {
        "feat_chsum": (o["feat"].sum(dim=(2, 3)), res["feat_chsum"]),
        "det_face_s8": (o["det"], res["det_face_s8"]),
        "det_face_s0": (o0, res["det_face_s0"]),
        "heatmaps": (o["heatmaps"], res["heatmaps"]),
        "emb": (o["emb"], res["emb"]),
        "norm": (o["norm"], res["norm"]),
    }
    for k, (a, b) in checks.items():
        d = float((a - b).abs().max())
        print(f"oracle vs reference {k}: max|d| = {d:.3e}")
        assert d <= 1e-4 * max(1.0, float(b.abs().max())), k

    meta = {
        "input_sum": np.float64(x.double().sum()),
        "w_resnet_conv1_sum": np.float64(sd["backbone.conv1.weight"].double().sum()),
        "w_vit_fc1_sum": np.float64(sd["vit_pose.vit_pose.backbone.encoder.layer.5.mlp.fc1.weight"].double().sum()),
        "bn_rv_sum": np.float64(sd["ada_face.adaface_model.body.10.res_layer.2.running_var"].double().sum()),
    }
    np.savez_compressed(os.path.join(GOLD, "golden_model.npz"),
                        **{k: v.numpy().astype(np.float32) for k, v in res.items()}, **meta)

    # ---- NMS (yolopt/util.py:123-169) on three inputs
    nms = reference_nms()
    gold = {}
    det = res["det_face_s8"]
    cases = {
        "det": det,                                  # [B,5,525] correct layout
        # what validation_step really feeds NMS: zero-stride head output (modify_yolo default)
        # transposed to [B,525,5] (module_v2.py:474-477)
        "evalstep": res["det_face_s0"].transpose(1, 2).contiguous(),
        "stress": nms_stress_input(),
    }
    for name, inp in cases.items():
        with torch.no_grad():
            dets = nms(inp.clone())
            mine = R.non_max_suppression(inp.clone())
        for a, b in zip(dets, mine):
            if name == "evalstep":
                # multi-label path (nc=521): exact score ties occur; the reference's tie order
                # is unspecified (unstable torch CPU sort) -> compare as row multisets
                assert a.shape == b.shape and torch.equal(_rowsort(a), _rowsort(b)), name
            else:
                assert a.shape == b.shape and torch.equal(a, b), name
        packed, cnt = _pack_dets(dets)
        gold[f"{name}_in"] = inp.numpy()
        gold[f"{name}_out"] = packed
        gold[f"{name}_count"] = cnt
        print(f"nms {name}: counts {cnt.tolist()}")
    np.savez_compressed(os.path.join(GOLD, "golden_nms.npz"), **gold)

    # ---- soft-argmax (pose_estimation/module.py:237-296)
    sa = reference_softargmax()
    hm2 = peaky_heatmaps()
    boxes = synth.uniform(11, "boxes", (3, 4)) * 200
    boxes[:, 2:] += boxes[:, :2] + 10
    g = {"model_in": res["heatmaps"].numpy(), "peaky_in": hm2.numpy(), "peaky_boxes": boxes.numpy()}
    for name, hm, bx in (("model", res["heatmaps"], None), ("peaky", hm2, boxes)):
        c, s = sa(hm.clone(), bx)
        c2, s2 = R.keypoints_from_heatmaps(hm.clone(), bx)
        assert torch.allclose(c, c2, atol=1e-6) and torch.allclose(s, s2, atol=1e-7), name
        g[f"{name}_coords"] = c.numpy()
        g[f"{name}_scores"] = s.numpy()
    np.savez_compressed(os.path.join(GOLD, "golden_softargmax.npz"), **g)
    for f in sorted(os.listdir(GOLD)):
        print(f, os.path.getsize(os.path.join(GOLD, f)))


if __name__ == "__main__":
    main()
