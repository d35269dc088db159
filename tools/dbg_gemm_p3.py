"""Debug (GPU box): GEMM-kernel precision 3 vs wave kernel vs fp64 on one small shape."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd"), os.path.join(ROOT, "tests")]
import torch
from test_gpu_ops import rnd, _g, _conv_p3, ref_conv
from prpe._lib import RES_PRE
for (B, Ci, H, W, Co, mags) in [(2, 64, 13, 11, 256, [1.0, 1.0]), (2, 64, 13, 11, 256, [7.0, 0.01]), (1, 64, 16, 16, 128, [1.0])]:
    x = torch.relu(rnd(B, Ci, H, W, seed=195)) * torch.tensor(mags).view(B, 1, 1, 1)
    w = rnd(Co, Ci, 1, 1, seed=196, scale=1.0 / math.sqrt(Ci))
    sc = torch.rand(Co, generator=_g(197)) + 0.5
    bi = rnd(Co, seed=198)
    ref = ref_conv(x, w, 1, 0, act="none", scale=sc, bias=bi)
    for t in (40, 42, 41, 27):
        try:
            y, _ = _conv_p3(x, w, 1, 0, tile=t, scale=sc, bias=bi, act="none")
        except Exception as e:
            print(t, "n/a", e); continue
        d = (y.double() - ref).abs()
        print(B, Ci, H, W, Co, mags, "tile", t, "max err", float(d.max()), "at", [int(v) for v in torch.nonzero(d == d.max())[0]])
