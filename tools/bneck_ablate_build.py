"""Build the fused-bottleneck ablation libraries (container; measurement only, results WRONG by
design) for tools/bneck_ablate.sh: each variant is a scratch copy of csrc/conv_bneck.hip with
parts of the kernel compiled out, compiled to an object and linked with the current build's
other objects and its build_info.o (same source hash, so prpe._lib loads it on the box).

    python tools/bneck_ablate_build.py [K ...]    # -> tools/abl/libprpe_ablK.so (default 4 5 6 7)

variants (round 4 had 1-4; round 5 adds 5-7 for the weight stream):
  1  phase-2 (3x3) MFMAs out          2  phase-1 MFMAs out        3  phase-3 MFMAs out
  4  every MFMA out (the data-movement skeleton)
  5  every MFMA AND the W1 / W2 / W3 LDS-DMA pieces out (the skeleton without the weight stream)
  6  the W1 / W2 / W3 LDS-DMA pieces out, MFMAs kept (they read stale LDS)
  7  every MFMA and the phase-1 x loads out (the skeleton without the haloed activation reads)
Run after person-recognition-for-pose-estimation_amd/build.py (it reuses build/*.o).
"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "build")
OUT = os.path.join(ROOT, "tools", "abl")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
         "-Wno-unused-result"]

MFMA = {  # phase -> the MFMA statement(s) of that phase in conv_bneck.hip
    1: ["acc2[j] = mfma3t(b, a, acc2[j]);"],
    2: ["acc1[0][j] = mfma3t(b, af[0], acc1[0][j]);", "if (two) acc1[1][j] = mfma3t(b, af[1], acc1[1][j]);"],
    3: ["acc3[j] = mfma3t(b, a, acc3[j]);"],
}
WDMA = ["bl_lds16(l ? wq1 : wq0, lds + bdst[i] + stage * STAGE, vo, kt * BK_ * 2);",
        "bl_lds16(q ? wr[2][1] : wr[2][0], w3b + ks * W3_STEP + (q * R3 + rb * 16) * 64, vo, ks * BK_ * 2);"]
XLOAD = ["raw[kt & 1][i][0] = bl_f4(xr, av[i], kt * BK_ * 4);", "raw[kt & 1][i][1] = bl_f4(xr, av[i] + 16, kt * BK_ * 4);"]

VARIANTS = {1: ([1], False, False), 2: ([2], False, False), 3: ([3], False, False), 4: ([1, 2, 3], False, False),
            5: ([1, 2, 3], True, False), 6: ([], True, False), 7: ([1, 2, 3], False, True)}


def patch(src, phases, wdma, xload):
    for ph in phases:
        for stmt in MFMA[ph]:
            assert stmt in src, stmt
            src = src.replace(stmt, "/* ablated */")
    if wdma:
        for stmt in WDMA:
            assert stmt in src, stmt
            src = src.replace(stmt, "(void)vo; /* ablated */")
    if xload:
        for stmt in XLOAD:
            assert stmt in src, stmt
            src = src.replace(stmt, "/* ablated */")
    return src


def main():
    os.makedirs(OUT, exist_ok=True)
    others = [o for o in glob.glob(os.path.join(BUILD, "*.o")) if not o.endswith("conv_bneck.o")]
    assert any(o.endswith("build_info.o") for o in others), "run build.py first"
    src0 = open(os.path.join(CSRC, "conv_bneck.hip")).read()
    want = [int(v) for v in sys.argv[1:]] or [4, 5, 6, 7]
    for k in want:
        phases, wdma, xload = VARIANTS[k]
        s = patch(src0, phases, wdma, xload)
        tmp = os.path.join(OUT, f"conv_bneck_abl{k}.hip")
        open(tmp, "w").write(s)
        obj = tmp[:-4] + ".o"
        r = subprocess.run([HIPCC, *FLAGS, "-c", tmp, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            sys.exit(f"variant {k}: {r.stderr[-2000:]}")
        lib = os.path.join(OUT, f"libprpe_abl{k}.so")
        r = subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *others, obj, "-o", lib],
                           capture_output=True, text=True)
        if r.returncode:
            sys.exit(f"link {k}: {r.stderr[-2000:]}")
        os.remove(obj)
        print("built", os.path.relpath(lib, ROOT), flush=True)


if __name__ == "__main__":
    main()
