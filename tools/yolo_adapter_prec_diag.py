"""Diagnostic (GPU box): which face-YOLO adapter layer carries the box error of policy "auto".
Planes handoff off (fp32 activations) so single layers can run at precision 2; each line raises
one adapter layer to precision 2 and reports the box / score error against the fp64 oracle on
the golden frames (bs=2).

    python tools/yolo_adapter_prec_diag.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

import torch  # noqa: E402

from oracle import model_ref as R  # noqa: E402
from prpe import CombinedModel, arch, engine, synth  # noqa: E402

RAISE = set()
_conv, _upconv = engine.Engine.conv, engine.Engine.upconv


def conv(self, x, p, *a, **k):
    if any(p.name.endswith(s) for s in RAISE):
        saved, self.precision = self.precision, 2
        try:
            return _conv(self, x, p, *a, **k)
        finally:
            self.precision = saved
    return _conv(self, x, p, *a, **k)


def upconv(self, name, *a, **k):
    if any((name + ":taps").endswith(s) or name.endswith(s) for s in RAISE):
        saved, self.precision = self.precision, 2
        try:
            return _upconv(self, name, *a, **k)
        finally:
            self.precision = saved
    return _upconv(self, name, *a, **k)


def main():
    torch.set_num_threads(16)
    engine.PLANES_ON = False
    engine.Engine.conv, engine.Engine.upconv = conv, upconv
    sd = synth.make_state_dict(arch.state_dict_spec())
    x = synth.frames(2)
    sd64 = {k: (v.double() if torch.is_floating_point(v) else v) for k, v in sd.items()}
    with torch.no_grad():
        f64 = R.resnet50_trunk(sd64, x.double())
        d64 = R.yolo_branch(sd64, "yolo_face", f64, [8.0, 16.0, 32.0])
    m = CombinedModel(sd, device="cuda")
    e = m.engine
    feat = e.trunk(x.cuda())
    a = "yolo_face.adapter"
    for layers in ([], [".0"], [".4"], [".7"], [".10"], [".13"], [".16"], [".0", ".4", ".7", ".10", ".13", ".16"]):
        RAISE.clear()
        RAISE.update(a + s for s in layers)
        det = e.yolo("yolo_face", feat, [8.0, 16.0, 32.0]).cpu().double()
        print(f"precision 2 on {layers}: box max|d| {(det[:, :4] - d64[:, :4]).abs().max().item():.3f} "
              f"cls {(det[:, 4] - d64[:, 4]).abs().max().item():.2e}", flush=True)


if __name__ == "__main__":
    main()
