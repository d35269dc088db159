"""CPU: the oracle (oracle/model_ref.py) against golden vectors produced by the reference
itself (oracle/make_golden.py, reference classes imported in the build container).

These pin the oracle; the GPU parity tests then compare the HIP path with the oracle and
with the same golden vectors."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

from oracle import model_ref as R
from prpe import synth


def _load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_synthetic_generators_are_the_golden_ones(state_dict, golden_model):
    x = synth.frames(2)
    assert float(x.double().sum()) == pytest.approx(float(golden_model["input_sum"]), rel=0, abs=1e-6)
    sd = state_dict
    assert float(sd["backbone.conv1.weight"].double().sum()) == float(golden_model["w_resnet_conv1_sum"])
    assert float(sd["vit_pose.vit_pose.backbone.encoder.layer.5.mlp.fc1.weight"].double().sum()) == \
        float(golden_model["w_vit_fc1_sum"])
    assert float(sd["ada_face.adaface_model.body.10.res_layer.2.running_var"].double().sum()) == \
        float(golden_model["bn_rv_sum"])


@pytest.fixture(scope="module")
def oracle_out(state_dict):
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    x = synth.frames(2)
    with torch.no_grad():
        o = R.forward_all(state_dict, x)
        o["det_s0"] = R.yolo_branch(state_dict, "yolo_face", o["feat"], (0.0, 0.0, 0.0))
        o["det_person_s0"] = R.yolo_branch(state_dict, "yolo_person", o["feat"], (0.0, 0.0, 0.0))
    return o


@pytest.mark.parametrize("key,gkey,tol", [
    ("det", "det_face_s8", 1e-5), ("det_s0", "det_face_s0", 0.0), ("det_person_s0", "det_person_s0", 0.0),
    ("heatmaps", "heatmaps", 1e-5), ("emb", "emb", 1e-6), ("norm", "norm", 1e-5)])
def test_oracle_model_matches_reference(oracle_out, golden_model, key, gkey, tol):
    a = oracle_out[key].numpy()
    b = golden_model[gkey]
    assert a.shape == b.shape
    assert np.abs(a - b).max() <= tol


def test_oracle_trunk_matches_reference(oracle_out, golden_model):
    cs = oracle_out["feat"].sum(dim=(2, 3)).numpy()
    np.testing.assert_allclose(cs, golden_model["feat_chsum"], rtol=0, atol=1e-3)


def test_zero_stride_quirk_gives_zero_boxes(golden_model):
    # modify_yolo leaves Head.stride = zeros (nn.py:238) -> every eval box coordinate is 0
    assert np.all(golden_model["det_face_s0"][:, :4] == 0)


@pytest.mark.parametrize("case", ["det", "evalstep", "stress"])
def test_oracle_nms_matches_reference(case):
    g = _load("golden_nms.npz")
    dets = R.non_max_suppression(torch.from_numpy(g[f"{case}_in"]))
    for i, d in enumerate(dets):
        n = int(g[f"{case}_count"][i])
        assert d.shape[0] == n
        ref = g[f"{case}_out"][i, :n]
        if case == "evalstep":   # tie order unspecified upstream: compare row multisets
            a = d.numpy()
            a = a[np.lexsort(a.T[::-1])]
            ref = ref[np.lexsort(ref.T[::-1])]
            np.testing.assert_array_equal(a, ref)
        else:
            np.testing.assert_array_equal(d.numpy(), ref)


@pytest.mark.parametrize("case,boxes", [("model", False), ("peaky", True)])
def test_oracle_softargmax_matches_reference(case, boxes):
    g = _load("golden_softargmax.npz")
    hm = torch.from_numpy(g[f"{case}_in"])
    bx = torch.from_numpy(g["peaky_boxes"]) if boxes else None
    c, s = R.keypoints_from_heatmaps(hm, bx)
    np.testing.assert_allclose(c.numpy(), g[f"{case}_coords"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(s.numpy(), g[f"{case}_scores"], rtol=1e-6, atol=0)


def test_oks_delta_identity():
    c = torch.rand(3, 17, 2)
    assert R.oks_delta(c, c) == 0.0
    assert R.oks_delta(c, c + 0.01) > 0.0


def test_oracle_yolo_raw_frames_matches_reference(state_dict):
    """Config-2 micro-bench variant: the reference's yolo_face.yolo on raw
    640x640 frames (A = 8400, oracle/make_golden_yolo_raw.py) -- det tensor and, on its tie-free
    copy, yolopt NMS -- against the oracle."""
    g = _load("golden_yolo_raw.npz")
    x = synth.frames(2)
    assert float(x.double().sum()) == pytest.approx(float(g["input_sum"]), rel=0, abs=1e-6)
    with torch.no_grad():
        det = R.yolo_net(state_dict, "yolo_face", x, [8.0, 16.0, 32.0])
    assert det.shape == (2, 5, 8400)
    assert np.abs(det.numpy() - g["det"]).max() <= 1e-5
    dets = R.non_max_suppression(torch.from_numpy(g["det_tiefree"]))
    for i, d in enumerate(dets):
        n = int(g["nms_count"][i])
        assert d.shape[0] == n
        np.testing.assert_array_equal(d.numpy(), g["nms_out"][i, :n])
