"""Build an A/B library (container; measurement only): one csrc file taken from a git revision,
linked with the current build's other objects and its build_info.o (same source hash, so
prpe._lib loads it on the box in place of libprpe.so; tools/bneck_ablate.sh-style swap).

    python tools/rev_variant_build.py REV csrc/conv_bneck.hip TAG   # -> tools/abl/libprpe_TAG.so
    python tools/rev_variant_build.py WORK csrc/conv_halo.hip TAG --patch OLD NEW [--patch ...]
    python tools/rev_variant_build.py /tmp/variant.hip csrc/pointwise.hip TAG   # a scratch copy
        (WORK = the working tree's file; measurement variants; csrc files may be comma-separated)

Run after person-recognition-for-pose-estimation_amd/build.py (it reuses build/*.o).
"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")
BUILD = os.path.join(PKG, "build")
OUT = os.path.join(ROOT, "tools", "abl")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "include"),
         "-I" + os.path.join(PKG, "csrc"), "-Wno-unused-result"]


def main():
    rev, rels, tag = sys.argv[1:4]
    rest = sys.argv[4:]
    os.makedirs(OUT, exist_ok=True)
    patches = []
    while rest:
        assert rest[0] == "--patch" and len(rest) >= 3, "usage: --patch OLD NEW"
        patches.append((rest[1], rest[2]))
        rest = rest[3:]
    objs, stems = [], []
    for rel in rels.split(","):                 # several csrc files: comma-separated
        name = os.path.basename(rel)
        if rev == "WORK":
            src = open(os.path.join(PKG, rel)).read()
        elif os.path.isfile(rev):                 # a scratch copy of the file (one csrc file)
            src = open(rev).read()
        else:
            src = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:person-recognition-for-pose-estimation_amd/{rel}"],
                                 capture_output=True, text=True, check=True).stdout
        for old, new in patches:
            if old in src:
                src = src.replace(old, new)
        stem = name.rsplit(".", 1)[0]
        stems.append(stem)
        tmp = os.path.join(OUT, f"{stem}_{tag}.hip")
        open(tmp, "w").write(src)
        obj = tmp[:-4] + ".o"
        subprocess.run([HIPCC, *FLAGS, "-c", tmp, "-o", obj], check=True)
        os.remove(tmp)
        objs.append(obj)
    others = [o for o in glob.glob(os.path.join(BUILD, "*.o")) if os.path.basename(o)[:-2] not in stems]
    assert any(o.endswith("build_info.o") for o in others), "run build.py first"
    lib = os.path.join(OUT, f"libprpe_{tag}.so")
    subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *others, *objs, "-o", lib], check=True)
    for o in objs:
        os.remove(o)
    print("built", os.path.relpath(lib, ROOT))


if __name__ == "__main__":
    main()
