"""Per-conv-layer timing of one full forward_all at bs=B (HIP events around every
prpe_conv2d launch), sorted by time, with algorithmic TF/s. GPU box only.

    python tools/layer_profile.py [--batch 256] [--precision auto] [--top 40]
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--precision", default="auto")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    prec = a.precision if a.precision == "auto" else int(a.precision)
    sd = synth.make_state_dict(arch.state_dict_spec())
    m = CombinedModel(sd, precision=prec)
    e = m.engine
    e.prepare()
    x = synth.frames(a.batch).cuda()
    m.forward_all(x, face_stride=[8.0, 16.0, 32.0], concurrent=False)
    torch.cuda.synchronize()
    e.watch = set(e._packs.keys()) | {"backbone.conv1+maxpool"}
    # fused bottlenecks (Engine.bottleneck) are timed under the block name; their row shows conv2
    e.watch |= {f"backbone.layer{li}.{b}" for li, (_, n, _) in enumerate(arch.RESNET50_STAGES, 1)
                for b in range(n)}
    # the bilinear-upsample -> 3x3 rewrites' second stage (prpe_upconv3x3), by adapter
    e.watch |= {k.rsplit(":", 1)[0] + ":upconv" for k in e._packs if k.endswith(":taps")}
    e.events = {}
    e.up_events = {}
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    m.forward_all(x, face_stride=[8.0, 16.0, 32.0], concurrent=False)
    t1.record()
    torch.cuda.synchronize()
    total = t0.elapsed_time(t1)
    rows = []
    for name, evs in e.events.items():
        ms = sum(s.elapsed_time(f) for s, f, *_ in evs)
        fl = sum(2.0 * px * p.co * p.ci * p.kh * p.kw for _, _, px, p, *_ in evs)
        _, _, px, p, prc, *_ = evs[0]
        rows.append((ms, name, len(evs), fl, p, prc, px))
    rows.sort(reverse=True)
    conv_ms = sum(r[0] for r in rows)
    print(f"forward_all bs={a.batch}: {total:.2f} ms total, convs {conv_ms:.2f} ms ({100 * conv_ms / total:.1f}%)")
    print(f"{'ms':>8} {'%':>5} {'TF/s':>7} prec  shape                     name")
    for ms, name, n, fl, p, prc, px in rows[:a.top]:
        shape = f"{p.kh}x{p.kw}/{p.stride} {p.ci}->{p.co} M={px}"
        print(f"{ms:8.3f} {100 * ms / total:5.1f} {fl / ms / 1e9:7.1f}  {prc}   {shape:26s} {name} x{n}")
    by = {}
    for ms, name, *_ in rows:
        comp = name.split(".")[0] if not name.startswith("vit") else "vit_pose"
        if name.startswith("ir50"):
            comp = "ada_face"
        by[comp] = by.get(comp, 0.0) + ms
    print("by component:", {k: round(v, 2) for k, v in sorted(by.items(), key=lambda t: -t[1])})
    # upconvs: time, and the rate of their output writes (the bound: z reads are small and L2-hot)
    up = []
    for name, evs in e.up_events.items():
        ms = sum(s.elapsed_time(f) for s, f, *_ in evs)
        yb = sum(ev[2] for ev in evs)
        zb = sum(ev[3] for ev in evs)
        up.append((ms, name, len(evs), yb, zb, evs[0][4], evs[0][5]))
    up.sort(reverse=True)
    print(f"upconvs (prpe_upconv3x3): {sum(u[0] for u in up):.3f} ms in total")
    for ms, name, n, yb, zb, pl, act in up:
        print(f"{ms:8.3f}  y {yb / 1e9:6.2f} GB -> {yb / ms / 1e9:6.2f} TB/s of writes  (z {zb / 1e9:5.2f} GB)  "
              f"{'planes' if pl else 'fp32'} {act:5s} {name} x{n}")


if __name__ == "__main__":
    main()
