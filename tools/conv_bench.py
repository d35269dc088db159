"""Micro-benchmark of prpe_conv2d on the model's heaviest conv shapes (GPU box).

    python tools/conv_bench.py [--batch 32] [--only NAME] [--prec 0,2] [--tiles 0]

Prints per (shape, precision, tile): mean ms, algorithmic TF/s, executed TF/s (x MFMA passes).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

import torch  # noqa: E402

from prpe import ops, pack  # noqa: E402

# name: (H, W, Ci, Co, k, stride, pad, frames-per-batch multiplier)
SHAPES = {
    "vit_adapter.7 3x3 256->128 @256x192": (256, 192, 256, 128, 3, 1, 1),
    "yolo_adapter.7 1x1 512->256 @160": (160, 160, 512, 256, 1, 1, 0),
    "yolo_adapter.10 3x3 256->128 @160": (160, 160, 256, 128, 3, 1, 1),
    "trunk l1 3x3 64->64 @160": (160, 160, 64, 64, 3, 1, 1),
    "trunk l1 1x1 64->256 @160": (160, 160, 64, 256, 1, 1, 0),
    "trunk l1 conv3 1x1 64->256 +res @160": (160, 160, 64, 256, 1, 1, 0, "res"),
    "trunk stem 7x7/2 4->64 @640": (640, 640, 4, 64, 7, 2, 3),
    "trunk l1 1x1 256->64 @160": (160, 160, 256, 64, 1, 1, 0),
    "trunk l3 3x3 256->256 @40": (40, 40, 256, 256, 3, 1, 1),
    "trunk l4 3x3 512->512 @20": (20, 20, 512, 512, 3, 1, 1),
    "trunk l3 1x1 1024->256 @40": (40, 40, 1024, 256, 1, 1, 0),
    "vit fc1 768->3072 (192 tok)": (16, 12, 768, 3072, 1, 1, 0),
    "vit fc2 3072->768 (192 tok)": (16, 12, 3072, 768, 1, 1, 0),
    "ada_adapter.7 3x3 256->128 @112": (112, 112, 256, 128, 3, 1, 1),
    "vit_adapter.10 3x3 128->3 @256x192": (256, 192, 128, 3, 3, 1, 1),
    "ir50 body 3x3 256->256 @14": (14, 14, 256, 256, 3, 1, 1),
    "vit qkv 768->2304 (192 tok)": (16, 12, 768, 2304, 1, 1, 0),
    "vit proj 768->768 (192 tok)": (16, 12, 768, 768, 1, 1, 0),
    "yolo_adapter.16 3x3 64->3 @160": (160, 160, 64, 3, 3, 1, 1),
    "yolo_adapter.13 1x1 128->64 @160": (160, 160, 128, 64, 1, 1, 0),
    "ir50 output 7x7 512->512 @7 (M = frames)": (7, 7, 512, 512, 7, 1, 0),
    "ada_adapter.10 3x3 128->64 @112": (112, 112, 128, 64, 3, 1, 1),
    "ada body.0 3x3 64->64 @112": (112, 112, 64, 64, 3, 1, 1),
    "ir50 body 3x3 64->64 @56": (56, 56, 64, 64, 3, 1, 1),
    "ir50 body 3x3 128->128 @28": (28, 28, 128, 128, 3, 1, 1),
    "ir50 body 3x3 512->512 @7": (7, 7, 512, 512, 3, 1, 1),
    "trunk l2 conv3 1x1 128->512 +res @80": (80, 80, 128, 512, 1, 1, 0, "res"),
    "trunk l3 conv3 1x1 256->1024 +res @40": (40, 40, 256, 1024, 1, 1, 0, "res"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--only", default="")
    ap.add_argument("--prec", default="0,2")
    ap.add_argument("--tiles", default="0")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--korders", default="0,1", help="weight K orders to compare (1 = chunk-major)")
    ap.add_argument("--amax", action="store_true", help="also track max|y| (y_amax) in the epilogue")
    ap.add_argument("--act", default="relu", help="epilogue activation (relu, gelu, silu, prelu, none)")
    ap.add_argument("--y-planes", action="store_true",
                    help="output in the planes format (y_planes, precision 0), as the model's ViT fc1 / qkv")
    ap.add_argument("--planes", action="store_true",
                    help="input in the planes format (x_planes; precision 0, wave-row kernel)")
    ap.add_argument("--prologue", action="store_true",
                    help="BN prologue on the input (in_scale / in_bias: the IR-50 res_layer's first conv)")
    ap.add_argument("--taps", type=int, default=0,
                    help="epilogue 1x1 GEMM to this many channels (prpe_conv_desc.w2; y not written)")
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    for name, (H, W, Ci, Co, k, s, p, *flags) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        B = a.batch
        x = torch.rand(B, H, W, Ci, device=dev) * 2 - 1
        w = (torch.rand(Co, Ci, k, k) * 2 - 1) / (Ci * k * k) ** 0.5
        pks = {}
        for ko in [int(v) for v in a.korders.split(",")]:
            if ko == 1 and (k == 1 or Ci % 32):
                continue
            pro = dict(in_scale=torch.rand(Ci) + 0.5, in_bias=torch.rand(Ci) - 0.5) if a.prologue else {}
            pks[ko] = pack.pack_conv("b", w, s, p, dev, scale=torch.ones(Co), bias=torch.zeros(Co), act=a.act,
                                     k_order=ko, **pro)
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y = torch.empty(B, Ho, Wo, Co, device=dev)
        r = torch.rand(B, Ho, Wo, Co, device=dev) if "res" in flags else None
        fl = 2.0 * B * Ho * Wo * Co * Ci * k * k
        xa = x.abs().flatten(1).amax(1).contiguous()
        ya = torch.zeros(x.shape[0], device=dev) if a.amax else None
        for (ko, pk) in pks.items():
          for prec in [int(v) for v in a.prec.split(",")]:
            for tile in [int(v) for v in a.tiles.split(",")]:
                kw = dict(res=r, res_mode=1 if r is not None else 0, precision=prec, tile=tile, y_amax=ya,
                          x_amax=xa if prec in (3, 4) else None, x_planes=a.planes,
                          y_planes=a.y_planes and prec == 0)
                if a.taps:
                    kw["w2"] = torch.rand(a.taps, Co, device=dev) - 0.5
                    kw["y2"] = torch.empty(B, Ho, Wo, a.taps, device=dev)
                try:
                    ops.conv2d(x, pk, y, **kw)
                except Exception as ex:              # tile not eligible for this shape
                    print(f"{name:40s} ko={ko} prec={prec} tile={tile}   n/a ({ex})", flush=True)
                    continue
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    ops.conv2d(x, pk, y, **kw)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                passes = {0: 3, 1: 1, 2: 6, 3: 3, 4: 1}[prec]
                tf = fl / ms / 1e9
                print(f"{name:40s} ko={ko} prec={prec} tile={tile} {ms:8.3f} ms  alg {tf:7.1f} TF/s  exec {tf * passes:7.1f} TF/s",
                      flush=True)


if __name__ == "__main__":
    main()
