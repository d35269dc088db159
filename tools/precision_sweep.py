"""Diagnostics (GPU box): parity vs the reference's golden outputs under several conv
precision policies (bs=2, 640x640)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]
import numpy as np, torch
from prpe import CombinedModel, arch, synth

g = dict(np.load(os.path.join(ROOT, "tests/golden/golden_model.npz")))
sd = synth.make_state_dict(arch.state_dict_spec())
x = synth.frames(2).cuda()
for name, pol in [("auto", "auto"), ("yolo_net=0", {"yolo_net": 0}), ("yolo all 2", {"yolo_adapter": 2}),
                  ("all 2", 2), ("all 0", 0)]:
    m = CombinedModel(sd, precision=pol)
    o = m.forward_all(x, face_stride=[8.0, 16.0, 32.0])
    d = o["det"].cpu().numpy(); r = g["det_face_s8"]
    print(f"{name:12s} cls {np.abs(d[:,4]-r[:,4]).max():.2e} box {np.abs(d[:,:4]-r[:,:4]).max():.2e} "
          f"heat {np.abs(o['heatmaps'].cpu().numpy()-g['heatmaps']).max():.2e} "
          f"emb {np.abs(o['emb'].cpu().numpy()-g['emb']).max():.2e}", flush=True)
