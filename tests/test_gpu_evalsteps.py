"""GPU: the eval-step kernels around the model against the oracle's
restatement of the reference code (oracle/model_ref.py: pose_flip_average restates
pose_estimation/module.py:476-484, face_recognition_eval restates face_recognition/module.py:
137-145). The reference runs these lines inline in Lightning validation steps, so no golden
vectors exist for them: parity is pinned to the restatement.

Tolerances: flip average bit-exact on the same heatmaps (same (a + b) * 0.5 in fp32); the
end-to-end flip test within the heatmap bar (1e-3 abs); cross-entropy within 1e-5 relative
(double-accumulated logsumexp vs torch's fp32), argmax exact except where the top-2 logits
of a row are closer than 1e-4 (fp32 GEMM rounding can swap a near-tie).
"""
import pytest
import torch

from oracle import model_ref as R
from prpe import CombinedModel, ops, synth
from prpe.evalsteps import FaceRecognitionEval, flip_partner, pose_flip_test

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["reference", "swap"])
def test_flip_average_bit_exact(mode):
    g = torch.Generator().manual_seed(5)
    heat = torch.rand(3, 17, 64, 48, generator=g)
    heat_f = torch.rand(3, 17, 64, 48, generator=g)
    got = ops.flip_average(heat.cuda(), heat_f.cuda(), flip_partner(17), 0 if mode == "reference" else 1)
    ref = R.pose_flip_average(heat, heat_f.clone(), mode)
    assert torch.equal(got.cpu(), ref)


def test_flip_average_rejects_bad_args():
    from prpe._lib import PrpeError
    h = torch.rand(1, 17, 4, 4, device="cuda")
    with pytest.raises(PrpeError):
        ops.flip_average(h, h, flip_partner(17), mode=2)
    with pytest.raises(PrpeError):
        ops.flip_average(h, h, [40] * 17, mode=0)


@pytest.fixture(scope="module")
def model(state_dict):
    return CombinedModel(state_dict, device="cuda")


def test_pose_flip_test_matches_explicit_flip(model):
    """the negative-stride mirrored read == running the model on torch.flip(frames)"""
    x = synth.frames(2).cuda()
    got = pose_flip_test(model, x, "reference")
    model.set_task("pose_estimation")
    h = model(x).heatmaps
    hf = model(torch.flip(x, dims=[-1]).contiguous()).heatmaps
    ref = R.pose_flip_average(h.cpu(), hf.cpu(), "reference")
    assert torch.equal(got.cpu(), ref)


def test_pose_flip_test_vs_oracle(model, state_dict):
    x = synth.frames(2)
    got = pose_flip_test(model, x.cuda(), "reference").cpu()
    with torch.no_grad():
        h = R.vitpose_branch(state_dict, R.resnet50_trunk(state_dict, x))
        hf = R.vitpose_branch(state_dict, R.resnet50_trunk(state_dict, torch.flip(x, dims=[-1])))
    ref = R.pose_flip_average(h, hf, "reference")
    assert (got - ref).abs().max().item() <= 1e-3


def test_ce_argmax_vs_torch():
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(37, 1000, generator=g) * 20
    logits[3, 10] = logits[3, 500] = 1e4           # tie: first index wins
    labels = torch.randint(0, 1000, (37,), generator=g)
    loss, amax, summary = ops.ce_argmax(logits.cuda(), labels.cuda())
    ref_rows = torch.nn.functional.cross_entropy(logits.double(), labels, reduction="none")
    torch.testing.assert_close(loss.cpu().double(), ref_rows, rtol=1e-6, atol=1e-5)
    assert torch.equal(amax.cpu().long(), logits.max(1)[1])
    assert amax[3].item() == 10
    s = summary.cpu()
    assert abs(s[0].item() - ref_rows.mean().item()) <= 1e-5 * max(1.0, ref_rows.mean().item())
    assert s[1].item() == (logits.max(1)[1] == labels).float().mean().item()


def test_face_recognition_eval_vs_oracle(model):
    g = torch.Generator().manual_seed(11)
    emb = torch.nn.functional.normalize(torch.randn(64, 512, generator=g))
    labels = torch.randint(0, 85742, (64,), generator=g)
    kernel = synth.head_kernel()
    model.ada_face.head.kernel = kernel.cuda()
    fr = FaceRecognitionEval(model, s=64.0)
    loss, acc, amax = fr(embeddings=emb.cuda(), labels=labels.cuda())
    rl, racc, rout, ramax = R.face_recognition_eval(emb, kernel, labels, 64.0)
    out = fr.logits(emb.cuda()).cpu()
    torch.testing.assert_close(out, rout, rtol=0, atol=2e-4)      # |logit| <= 64
    top2 = rout.topk(2, dim=1).values
    near_tie = (top2[:, 0] - top2[:, 1]) < 1e-4
    mism = amax.cpu().long() != ramax
    assert not torch.any(mism & ~near_tie)
    assert abs(loss.item() - rl.item()) <= 1e-4 * max(1.0, abs(rl.item()))
    if not torch.any(near_tie):
        assert acc.item() == racc.item()
