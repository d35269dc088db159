"""Static ISA summary of a HIP source's kernels (container, no GPU): VGPRs, scratch, and the
instruction mix of the innermost loops that hold MFMAs (per loop: MFMA / VALU / SALU / DS / VMEM).

    python tools/isa_loops.py person-recognition-for-pose-estimation_amd/csrc/conv_wave.hip [name-regex]
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
        meta = {k: None for k in ("NumVgprs", "ScratchSize", "Occupancy")}
        for l in body:
            for k in meta:
                m = re.search(rf"; {k}: (\d+)", l)
                if m:
                    meta[k] = int(m.group(1))
        cnt, hdr, blk = {}, {}, None
        for l in body:
            m = re.match(r"^(\.LBB\w+):\s*(;.*)?", l)
            if m:
                blk = m.group(1)
                cnt[blk] = [0] * 5
                c = m.group(2) or ""
                h = re.search(r"Header=BB(\w+) Depth=(\d)", c) or re.search(r"Loop Header: Depth=(\d)", c)
                hdr[blk] = ("BB" + blk[4:], None) if "=>This" in c else (("BB" + h.group(1)) if h and h.lastindex == 2 else None)
                continue
            t = l.strip()
            if blk is None or not t or t.startswith((".", ";")):
                continue
            k = 0 if t.startswith("v_mfma") else 1 if t.startswith("v_") else 2 if t.startswith("s_") else \
                3 if t.startswith("ds_") else 4 if t.startswith(("global_", "buffer_", "scratch_")) else None
            if k is not None:
                cnt[blk][k] += 1
        loops = {}
        for blk, h in hdr.items():
            key = h[0] if isinstance(h, tuple) else h
            if key:
                loops.setdefault(key, [0] * 5)
                loops[key] = [x + y for x, y in zip(loops[key], cnt[blk])]
        short = re.sub(r"^_ZN6prpe_k12_GLOBAL__N_1\d+", "", name)[:70]
        print(f"{short}  vgpr {meta['NumVgprs']} scratch {meta['ScratchSize']} occ {meta['Occupancy']}")
        for key, c in loops.items():
            if c[0]:
                print(f"    loop {key}: mfma {c[0]} valu {c[1]} salu {c[2]} ds {c[3]} vmem {c[4]}  "
                      f"valu/mfma {c[1] / c[0]:.2f}")


if __name__ == "__main__":
    main()
