"""Diagnostics (GPU box): stage-by-stage error of the HIP path vs the oracle, each branch fed
the ORACLE's trunk features so errors are isolated per stage; plus the oracle's own
sensitivity to 2^-17 relative weight noise (what split-bf16 rounding can cost at best)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import model_ref as R  # noqa: E402
from prpe import arch, synth  # noqa: E402
from prpe.engine import Engine  # noqa: E402


def err(name, a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    d = (a - b).abs()
    print(f"{name:40s} max|d|={d.max():.3e} mean|d|={d.mean():.3e} max|ref|={b.abs().max():.3e} "
          f"rel={d.max() / (b.abs().max() + 1e-30):.3e}", flush=True)


def main():
    torch.set_num_threads(16)
    sd = synth.make_state_dict(arch.state_dict_spec())
    x = synth.frames(1)
    with torch.no_grad():
        feat = R.resnet50_trunk(sd, x)
    e = Engine(sd, "cuda")
    g = e.trunk(x.cuda())
    err("trunk feat", g.permute(0, 3, 1, 2), feat)
    featd = feat.permute(0, 2, 3, 1).contiguous().cuda()

    # ---- ViT adapter + backbone
    with torch.no_grad():
        pix = R.vitpose_adapter(sd, feat)
        heat = R.vitpose_backbone(sd, pix)
    gp = e.vit_adapter(featd)
    err("vit adapter pixel_values", gp.permute(0, 3, 1, 2), pix)
    gh = e.vit_backbone(pix.permute(0, 2, 3, 1).contiguous().cuda())
    err("vit backbone heatmaps (oracle pix)", gh, heat)
    err("vit full branch heatmaps", e.vitpose(featd), heat)

    # ---- AdaFace
    with torch.no_grad():
        emb, norm = R.adaface_branch(sd, feat)
    ge, gn = e.adaface(featd)
    err("adaface emb", ge, emb)
    err("adaface norm", gn, norm)

    # ---- YOLO adapter
    a = "yolo_face.adapter"
    with torch.no_grad():
        t = F.silu(R._bn(sd, a + ".1", R._conv(sd, a + ".0", feat)))
        u = F.interpolate(t, size=(160, 160), mode="bilinear", align_corners=True)
        u = F.silu(R._bn(sd, a + ".5", R._conv(sd, a + ".4", u, 1, 1)))
        y = F.silu(R._bn(sd, a + ".8", R._conv(sd, a + ".7", u)))
        y = F.silu(R._bn(sd, a + ".11", R._conv(sd, a + ".10", y, 1, 1)))
        y = F.silu(R._bn(sd, a + ".14", R._conv(sd, a + ".13", y)))
        y = F.silu(R._bn(sd, a + ".17", R._conv(sd, a + ".16", y, 1, 1)))
        print("yolo adapter out per-channel std:", y.std(dim=(2, 3)).flatten().tolist())
        det = R.yolo_branch(sd, "yolo_face", feat, (8.0, 16.0, 32.0))
    gt = e.conv(featd, e.pk(a + ".0", a + ".0.weight", bn=a + ".1", bias_key=a + ".0.bias", act="silu"))
    err("yolo adapter.0", gt.permute(0, 3, 1, 2), t)
    gu = e.upconv(a + ".4", gt, a + ".4.weight", (160, 160), True, bn=a + ".5", bias_key=a + ".4.bias", act="silu")
    err("yolo adapter upconv", gu.permute(0, 3, 1, 2), u)
    gd = e.yolo("yolo_face", featd, (8.0, 16.0, 32.0))
    err("yolo det cls", gd[:, 4], det[:, 4])
    err("yolo det box", gd[:, :4], det[:, :4])

    # ---- intrinsic sensitivity: oracle with weights * (1 + 2^-17 * U(-1,1))
    g = torch.Generator().manual_seed(0)
    sdn = {}
    for k, v in sd.items():
        if v.dtype == torch.float32 and v.dim() >= 2:
            sdn[k] = v * (1 + (torch.rand(v.shape, generator=g) * 2 - 1) * 2 ** -17)
        else:
            sdn[k] = v
    with torch.no_grad():
        on = R.forward_all(sdn, x)
        o = R.forward_all(sd, x)
    for k in ("feat", "det", "emb", "norm", "heatmaps"):
        err(f"[sensitivity 2^-17 weights] {k}", on[k], o[k])


if __name__ == "__main__":
    main()
