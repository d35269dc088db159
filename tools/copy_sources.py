"""Where the device-to-device copies of a forward come from (GPU box, diagnostics): runs the full
bench step (forward_all + NMS + soft-argmax, bs from --batch) under torch.profiler with Python
stacks and prints the aten::copy_ / memcpy-issuing ops grouped by their innermost prpe frame.

    python tools/copy_sources.py --batch 64
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    import torch
    from prpe import CombinedModel, arch, ops, synth
    from prpe.postproc import non_max_suppression_padded
    dev = torch.device("cuda", 0)
    sd = synth.make_state_dict(arch.state_dict_spec())
    model = CombinedModel(sd, device=dev, precision="auto")
    model.engine.prepare()
    x = synth.frames(a.batch, seed=100).to(dev)

    def step():
        o = model.forward_all(x, face_stride=[8.0, 16.0, 32.0], concurrent=True)
        dets, cnt = non_max_suppression_padded(o["det"])
        ops.softargmax(o["heatmaps"])
        return dets, cnt

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    by = collections.Counter()
    for ev in prof.events():
        if ev.name not in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::cat", "aten::to", "aten::_to_copy"):
            continue
        frames = [f for f in (ev.stack or []) if "prpe" in f or "bench" in f or "model" in f]
        key = frames[0] if frames else "(no prpe frame)"
        by[(ev.name, key)] += 1
    print(f"# ops that can issue device copies in one bench step (bs={a.batch}), by innermost prpe frame")
    for (name, key), n in by.most_common(40):
        print(f"{n:5d}  {name:18s} {key}")


if __name__ == "__main__":
    main()
