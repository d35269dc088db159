"""Run one trunk launch in isolation (for rocprofv3 PMC passes): the stem (copy_pad + the
chunked 7x1/2 conv) or the layer1.0 conv3 + downsample dual-input GEMM, at precision 3 on
the model's own packs. GPU box only.

    python tools/trunk_kernels.py stem|dual [--batch 64] [--iters 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

import torch  # noqa: E402

from prpe import CombinedModel, arch, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["stem", "dual"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    sd = synth.make_state_dict(arch.state_dict_spec())
    e = CombinedModel(sd, precision="auto").engine
    B = a.batch
    x = synth.frames(B).cuda()
    if a.what == "stem":
        for _ in range(a.iters):
            with e.prec("trunk"):              # each entry zeroes the trunk's max|y| slots
                e.stem(x)
    else:
        with e.prec("trunk"):
            o = torch.relu(torch.randn(B, 160, 160, 64, device="cuda"))
            xs = torch.relu(torch.randn(B, 160, 160, 64, device="cuda"))
        o._prpe_amax = o.abs().flatten(1).amax(1).contiguous()
        xs._prpe_amax = xs.abs().flatten(1).amax(1).contiguous()
        for _ in range(a.iters):
            with e.prec("trunk"):
                e.conv(o, e.pk_dual("backbone.layer1.0"), x2=xs, x2_amax=xs._prpe_amax)
    torch.cuda.synchronize()
    print("ok", a.what, B)


if __name__ == "__main__":
    main()
