"""Static check of the conv main loops (container, no GPU): for every kernel in a HIP source,
print the s_waitcnt instructions the compiler placed between the last LDS-DMA issue and the
first MFMA of the K-step. A vmcnt there means the K-step waits for the loads it just issued
(the A prefetch and the B ring then no longer overlap the MFMAs).

    python tools/loop_waits.py person-recognition-for-pose-estimation_amd/csrc/conv_wave.hip [filter]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-I" + os.path.join(ROOT, "include"),
                        "-I" + os.path.join(ROOT, "person-recognition-for-pose-estimation_amd", "csrc"),
                        "--cuda-device-only", "-S", "-o", out, src], check=True, capture_output=True)
        lines = open(out).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)] + [len(lines)]
    for a, b in zip(starts, starts[1:]):
        name = lines[a].split(":")[0]
        if flt and not re.search(flt, name):
            continue
        body = lines[a:b]
        first = next((i for i, l in enumerate(body) if "mfma" in l), None)
        if first is None:
            continue
        dma = max((i for i, l in enumerate(body[:first]) if "global_load_lds" in l), default=None)
        lo = dma if dma is not None else max(0, first - 60)
        waits = [l.strip() for l in body[lo:first] if "s_waitcnt" in l]
        bad = any("vmcnt" in w for w in waits)
        print(("VMCNT " if bad else "ok    ") + f"{name[:90]:90s} {waits}")


if __name__ == "__main__":
    main()
