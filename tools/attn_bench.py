"""Micro-benchmark of prpe_attention (ViTPose-B: 192 tokens, 12 heads, d 64) at bs frames (GPU box).

    python tools/attn_bench.py [--batch 256] [--iters 10]

Prints ms per call, executed MFMA TF/s (3 split passes) and the K/V/Q/O bytes moved.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

import torch  # noqa: E402

from prpe import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    B, L, H, D = a.batch, 192, 12, 64
    qkv = torch.rand(B * L, 3 * H * D, device="cuda") - 0.5
    out = torch.empty(B * L, H * D, device="cuda")
    ops.attention(qkv, out, B, L, H, D, D ** -0.5)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ops.attention(qkv, out, B, L, H, D, D ** -0.5)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    fl = 4.0 * B * H * L * L * D
    by = 4.0 * B * L * H * D * 4
    print(f"attention bs={B}: {ms:.3f} ms  alg {fl / ms / 1e9:.1f} TF/s  exec {3 * fl / ms / 1e9:.1f} TF/s  "
          f"{by / ms / 1e6:.0f} GB/s (q,k,v read + o write)")


if __name__ == "__main__":
    main()
