"""Sequential forward_all passes at bs=B for kernel-trace profiling (GPU box):

    rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python tools/seq_forward.py [--batch 256] [--passes 2]

One untimed warm-up pass (weight packing, allocator), then `passes` sequential passes (heads
on one stream, so every launch's duration is its own, not shared with concurrent heads).
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
    ap.add_argument("--passes", type=int, default=2)
    a = ap.parse_args()
    m = CombinedModel(synth.make_state_dict(arch.state_dict_spec()))
    m.engine.prepare()
    x = synth.frames(a.batch).cuda()
    m.forward_all(x, face_stride=[8.0, 16.0, 32.0], concurrent=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.passes):
        m.forward_all(x, face_stride=[8.0, 16.0, 32.0], concurrent=False)
    e1.record()
    torch.cuda.synchronize()
    print(f"sequential forward_all bs={a.batch}: {e0.elapsed_time(e1) / a.passes:.2f} ms/pass", flush=True)


if __name__ == "__main__":
    main()
