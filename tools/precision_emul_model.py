"""CPU emulation (diagnostics, no GPU) of reduced-operand MFMA policies on the WHOLE model:
the oracle (oracle/model_ref.py, fp32) is re-run with the conv / linear operands of chosen
layer groups rounded the way a kernel would feed them to the MFMA, accumulation and storage
staying fp32. Reports heatmaps / embeddings / YOLO scores / boxes / OKS against the plain
fp32 oracle on the same frames.

    python tools/precision_emul_model.py [--frames 2] [policy ...]

Operand schemes (per layer group):
  f16    one fp16 plane each, RNE: weights scaled per output channel (max |w| in [2^14,2^15)),
         activations per FRAME (max |x| < 2^e -> x 2^(15-e)); 1 MFMA term
  f16a   activations one fp16 plane, weights two planes (exact to ~2^-22): 2 terms
  f16w   weights one plane, activations two planes: 2 terms
  bf16   one bf16 plane each (RNE): 1 term
  bf16x3 two bf16 planes each, 3 terms (today's precision 0)
  f16x3  two scaled fp16 planes each, 3 terms (precision 3)

    --seed N              weight seed of the synthetic net (prpe.synth; default its WEIGHT_SEED)
    --ada-gamma LO,HI     redraw the IR-50 residual-branch tail gammas (res_layer.5) from U(LO, HI)
                          instead of the tamed U(0.05, 0.25): the precision-4 robustness check of
                          round 5 (profiles/r05_precision4_robustness.txt)
For the upsample->conv3x3 layers the GPU's GEMM operand is the LOW-resolution tensor (tap
rewrite), so the activation rounding is applied before the interpolation.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import model_ref as R  # noqa: E402
from prpe import arch, synth  # noqa: E402


def _rne16(v):
    return v.to(torch.float16).float()


def _rbf(v):
    return v.to(torch.bfloat16).float()


def q_act(x, scheme):
    """x [B, ...] fp32 -> value the MFMA sees (per-frame scale)."""
    if scheme in ("f16", "f16a"):
        m = x.abs().flatten(1).amax(1)
        _, e = torch.frexp(m)
        e = torch.where(m > 0, e, torch.full_like(e, 15))
        s = torch.ldexp(torch.ones_like(m), 15 - e).view(-1, *([1] * (x.dim() - 1)))
        return _rne16(x * s) / s
    if scheme == "f16w":
        m = x.abs().flatten(1).amax(1)
        _, e = torch.frexp(m)
        s = torch.ldexp(torch.ones_like(m), 15 - e).view(-1, *([1] * (x.dim() - 1)))
        h = _rne16(x * s)
        return (h + _rne16(x * s - h)) / s
    if scheme == "bf16":
        return _rbf(x)
    if scheme == "bf16x3":
        h = _rbf(x)
        return h + _rbf(x - h)      # the 3-term product drops lo*lo: emulated at operand level
    if scheme == "f16x3":
        return q_act(x, "f16w")
    return x


def q_w(w, scheme):
    """w [co, ...] -> rounded weight (per output channel scale)."""
    if scheme in ("f16", "f16w"):
        m = w.abs().flatten(1).amax(1)
        _, e = torch.frexp(m)
        e = torch.where(m > 0, 15 - e, torch.zeros_like(e))
        s = torch.ldexp(torch.ones_like(m), e).view(-1, *([1] * (w.dim() - 1)))
        return _rne16(w * s) / s
    if scheme in ("f16a", "f16x3"):
        m = w.abs().flatten(1).amax(1)
        _, e = torch.frexp(m)
        e = torch.where(m > 0, 15 - e, torch.zeros_like(e))
        s = torch.ldexp(torch.ones_like(m), e).view(-1, *([1] * (w.dim() - 1)))
        h = _rne16(w * s)
        return (h + _rne16(w * s - h)) / s
    if scheme == "bf16":
        return _rbf(w)
    if scheme == "bf16x3":
        h = _rbf(w)
        return h + _rbf(w - h)
    return w


GROUPS = {
    "trunk": lambda p: p.startswith("backbone."),
    "trunk_l3": lambda p: p.startswith("backbone.layer3"),
    "trunk_l4": lambda p: p.startswith("backbone.layer4"),
    "trunk_l12": lambda p: p.startswith("backbone.layer1") or p.startswith("backbone.layer2"),
    "yolo_adapter": lambda p: ".adapter." in p and p.startswith("yolo_"),
    "yolo_net": lambda p: p.startswith("yolo_") and ".yolo." in p,
    "ada_adapter": lambda p: p.startswith("ada_face.adapter."),
    "ir50": lambda p: p.startswith("ada_face.adaface_model."),
    "vit_adapter": lambda p: p.startswith("vit_pose.adapter."),
    "vit_patch": lambda p: "patch_embeddings" in p,
    "vit_qkv": lambda p: ".attention.attention." in p,
    "vit_proj": lambda p: ".attention.output." in p,
    "vit_fc1": lambda p: ".mlp.fc1" in p,
    "vit_fc2": lambda p: ".mlp.fc2" in p,
    "vit_head": lambda p: p.startswith("vit_pose.vit_pose.head"),
    "vit_a7": lambda p: p.startswith("vit_pose.adapter.7"),          # the dominant 3x3 alone
    "yolo_a10": lambda p: p.startswith("yolo_face.adapter.10"),
    "yolo_a7": lambda p: p.startswith("yolo_face.adapter.7"),
    "ada_a7": lambda p: p.startswith("ada_face.adapter.7"),
}
UPCONV = ("yolo_face.adapter.4", "yolo_person.adapter.4", "ada_face.adapter.4", "vit_pose.adapter.4",
          "vit_pose.vit_pose.head.conv")


class Emul:
    def __init__(self, policy: dict):
        self.policy = policy
        self.pending_up = None        # scheme to apply at the next interpolate

    def scheme(self, p):
        for g, s in self.policy.items():
            if GROUPS[g](p):
                return s
        return None

    def install(self):
        orig_conv = R._conv
        orig_linear = F.linear
        orig_interp = F.interpolate
        em = self
        wmap = {}

        def conv(sd, p, x, stride=1, padding=0, groups=1):
            s = em.scheme(p)
            if s is None or groups != 1:
                return orig_conv(sd, p, x, stride, padding, groups)
            w = sd[p + ".weight"]
            if p in UPCONV:
                xq = x                # rounded before the interpolation
            else:
                xq = q_act(x, s)
            return F.conv2d(xq, q_w(w, s), sd.get(p + ".bias"), stride, padding, 1, groups)

        def interp(x, *a, **k):
            s = em.pending_up
            if s is not None and k.get("mode") == "bilinear":
                x = q_act(x, s)
            return orig_interp(x, *a, **k)

        sd_ref = {}

        def linear(x, w, b=None):
            p = wmap.get(id(w))
            s = em.scheme(p) if p else None
            if s is None:
                return orig_linear(x, w, b)
            B = x.shape[0]
            xq = q_act(x.reshape(B, -1), s).reshape(x.shape) if x.dim() > 2 else q_act(x, s)
            return orig_linear(xq, q_w(w, s), b)

        self.wmap = wmap
        self.sd_ref = sd_ref
        R._conv = conv
        F.linear = linear
        F.interpolate = interp
        # the ViT patch-embed / decoder conv call F.conv2d directly in the oracle: route them
        orig_conv2d = F.conv2d

        def conv2d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
            p = wmap.get(id(w))
            s = em.scheme(p) if p else None
            if s is None or groups != 1:
                return orig_conv2d(x, w, b, stride, padding, dilation, groups)
            xq = x if p in UPCONV else q_act(x, s)
            return orig_conv2d(xq, q_w(w, s), b, stride, padding, dilation, groups)

        F.conv2d = conv2d
        self._orig = (orig_conv, orig_linear, orig_interp, orig_conv2d)

    def uninstall(self):
        R._conv, F.linear, F.interpolate, F.conv2d = self._orig

    def register(self, sd):
        for k, v in sd.items():
            if k.endswith(".weight") and v.dim() >= 2:
                self.wmap[id(v)] = k[: -len(".weight")]


def run_policy(sd, x, policy):
    em = Emul(policy)
    em.install()
    em.register(sd)
    try:
        # interpolate rounding: set per branch by peeking at the upconv layer's group
        def hook_branch(fn, up_prefix):
            def w(*a, **k):
                em.pending_up = em.scheme(up_prefix)
                try:
                    return fn(*a, **k)
                finally:
                    em.pending_up = None
            return w
        yb, ab, va, vb = R.yolo_branch, R.adaface_branch, R.vitpose_adapter, R.vitpose_backbone
        R.yolo_branch = lambda sd_, p, *a, **k: hook_branch(yb, p + ".adapter.4")(sd_, p, *a, **k)
        R.adaface_branch = hook_branch(ab, "ada_face.adapter.4")
        R.vitpose_adapter = hook_branch(va, "vit_pose.adapter.4")
        R.vitpose_backbone = hook_branch(vb, "vit_pose.vit_pose.head.conv")
        try:
            with torch.no_grad():
                return R.forward_all(sd, x)
        finally:
            R.yolo_branch, R.adaface_branch, R.vitpose_adapter, R.vitpose_backbone = yb, ab, va, vb
    finally:
        em.uninstall()


def parse_policy(s):
    if s == "fp32":
        return {}
    pol = {}
    for part in s.split(","):
        g, sch = part.split("=")
        gs = list(GROUPS) if g == "all" else ([k for k in GROUPS if k.startswith("vit_")] if g == "vit" else [g])
        for k in gs:
            pol[k] = sch
    return pol


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--ada-gamma", default=None)
    ap.add_argument("policies", nargs="*", default=["all=bf16x3", "all=f16"])
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    seed = synth.WEIGHT_SEED if a.seed is None else a.seed
    sd = synth.make_state_dict(arch.state_dict_spec(), seed=seed)
    if a.ada_gamma:
        lo, hi = (float(v) for v in a.ada_gamma.split(","))
        n = 0
        for k in list(sd):
            if k.startswith("ada_face.adaface_model.") and k.endswith("res_layer.5.weight"):
                sd[k] = synth.uniform(seed + 7, k, tuple(sd[k].shape), lo, hi)
                n += 1
        print(f"# IR-50 residual-branch gammas redrawn from U({lo}, {hi}): {n} tensors", flush=True)
    print(f"# weight seed {seed}, {a.frames} frames", flush=True)
    x = synth.frames(a.frames)
    with torch.no_grad():
        ref = R.forward_all(sd, x)
    rc, _ = R.keypoints_from_heatmaps(ref["heatmaps"])
    rb = ref["det"][:, :4].abs().max()
    for s in a.policies:
        t0 = time.time()
        o = run_policy(sd, x, parse_policy(s))
        c, _ = R.keypoints_from_heatmaps(o["heatmaps"])
        print(f"{s:60s} heat {float((o['heatmaps'] - ref['heatmaps']).abs().max()):.2e} "
              f"emb {float((o['emb'] - ref['emb']).abs().max()):.2e} "
              f"emb-norm/rel {float(((o['norm'] - ref['norm']).abs() / ref['norm'].abs()).max()):.1e} "
              f"cls {float((o['det'][:, 4] - ref['det'][:, 4]).abs().max()):.2e} "
              f"box/max {float((o['det'][:, :4] - ref['det'][:, :4]).abs().max() / rb):.2e} "
              f"oks {R.oks_delta(c, rc):.1e}  ({time.time() - t0:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
