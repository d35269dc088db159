"""Micro-bench (GPU box): the fused identity bottleneck (prpe_bottleneck) vs the three unfused
precision-3 launches on the layer1 shape [B, 160, 160, 256], random post-ReLU input; with
--proj the projection block (layer1.0: x [B, 160, 160, 64], conv3 + downsample as one dual GEMM).

    python tools/bneck_bench.py --batch 256 --iters 10 [--fused-only] [--proj]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from prpe import ops  # noqa: E402

DEV = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--fused-only", action="store_true")
    ap.add_argument("--proj", action="store_true")
    ap.add_argument("--mid", type=int, default=64, help="128: layer2's identity block [B, 80, 80, 512]")
    a = ap.parse_args()
    from test_gpu_bneck import _packs, _packs128, _packs_proj, _unfused, _unfused128, _unfused_proj  # noqa: E402
    if a.mid == 128:
        _, _, packs = _packs128(600)
        unfused, cin, cout, hw = _unfused128, 512, 512, 80
    else:
        _, _, packs = _packs_proj(500) if a.proj else _packs(400)
        unfused = _unfused_proj if a.proj else _unfused
        cin, cout, hw = (64 if a.proj else 256), 256, 160
    g = torch.Generator(DEV).manual_seed(1)
    x = torch.relu(torch.randn(a.batch, hw, hw, cin, generator=g, device=DEV))
    xa = x.abs().flatten(1).amax(1).contiguous()
    y = torch.empty(a.batch, hw, hw, cout, device=DEV)
    ya = torch.zeros(a.batch, device=DEV)
    px = a.batch * hw * hw
    gb = px * (cin + cout) * 4 / 1e9               # algorithmic: x read once, y written once

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    ms = timed(lambda: ops.bottleneck(x, packs, y, xa, ya))
    print(f"{'proj ' if a.proj else ''}mid {a.mid} fused   bs={a.batch}: {ms:.3f} ms  {gb / ms:.2f} TB/s algorithmic ({gb:.2f} GB)", flush=True)
    if not a.fused_only:
        ms_u = timed(lambda: unfused(x, xa, packs))
        print(f"unfused bs={a.batch}: {ms_u:.3f} ms (three launches)", flush=True)


if __name__ == "__main__":
    main()
