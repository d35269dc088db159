"""VGPR / AGPR / spill / LDS usage of every kernel in a HIP source (container: compiles the
device code to assembly and reads the AMDHSA metadata).

    python tools/kernel_resources.py person-recognition-for-pose-estimation_amd/csrc/conv_wave.hip [filter]
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
        s = open(out).read()
    for blk in re.findall(r"- \.agpr_count:.*?\.wavefront_size", s, re.S):
        get = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
        name = get("name")
        if flt and not re.search(flt, name):
            continue
        print(f"vgpr {get('vgpr_count'):>4} agpr {get('agpr_count'):>3} spill {get('vgpr_spill_count'):>3} "
              f"lds {get('group_segment_fixed_size'):>6}  {name}")


if __name__ == "__main__":
    main()
