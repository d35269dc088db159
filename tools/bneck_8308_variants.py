"""Round-5 root-cause experiment for the reverted commit 8308d2f (fused bottleneck reading conv3's
scale / bias from an LDS-DMA'd copy in ring stage 3; on the GPU its layer1 identity blocks gave
garbage that differed run to run). Container side: writes variants of THAT
commit's conv_bneck.hip (git show 8308d2f) and links each with the current build's other
objects into tools/abl/libprpe_8308<X>.so for tools/bneck_8308.sh (GPU box, test_gpu_bneck.py
on each in turn). Measurement only: none of these ship.

  A  8308d2f as committed
  B  A + s_waitcnt vmcnt(0) right after each issue_w3(h + 1): the W3 LDS-DMA pieces have landed
     before the part's y stores and the next part's residual loads are issued
  C  A with the SB3 copy issued by EVERY wave (identical bytes), so every wave's vmcnt history is
     the same
  D  A + s_waitcnt vmcnt(0) after each part's y stores (before the next part's residual loads):
     the W3 pieces land before the residual loads are issued, the stores are drained too
  (round 5, second batch -- A-D all failed identically, so not an ordering race; what fails is
   exactly the kernels whose phase-1 tile-max slots (wmax1, ring stage (NK1 - 1) % 4) sit at the
   SB3 address: identity mid 64 (NK1 = 8) and mid 128 (NK1 = 16) use stage 3, the passing
   projection block (NK1 = 2) stage 1)
  E  A with SB3 at ring stage 2 + 1 KiB (past the phase-3 tile-max slots; no phase-1 access there)
  F  A with the phase-1 tile-max slots moved to ring stage 2 + 4 KiB (away from SB3)
  G  A with SB3 filled by register staging (global loads + ds_write) instead of LDS-DMA
  (third batch -- E and G failed exactly as A, F worse: neither the copy mechanism nor its place)
  J  A with the epilogue reading scale / bias from global memory again (the SB3 copy still made,
     unused): does the copy corrupt anything, or is it the epilogue's LDS read?
  K  A with the epilogue's bias from global memory, the scale from LDS
  L  A with the epilogue's scale from global memory, the bias from LDS
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


def variants(src):
    out = {"A": src}
    w3 = "issue_w3(h + 1);"
    assert src.count(w3) == 2
    out["B"] = src.replace(w3, 'issue_w3(h + 1); asm volatile("s_waitcnt vmcnt(0)" ::: "memory");')
    old = "    if (wave < 2 * NSB) {\n      const int arr = wave / NSB, pc = wave % NSB;"
    assert old in src
    out["C"] = src.replace(old, "    {\n      const int arr = (wave / NSB) & 1, pc = wave % NSB;")
    st = "      bs_f4(yr, v, yvo, (h * R3 + j * 16) * 4);\n    }\n"
    assert src.count(st) == 1
    out["D"] = src.replace(st, st + '    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n')
    sb = "  constexpr int SB3_OFF = RING_OFF + 3 * STAGE;"
    assert sb in src
    out["E"] = src.replace(sb, "  constexpr int SB3_OFF = RING_OFF + 2 * STAGE + 1024;")
    wm = "reinterpret_cast<float*>(lds + RING_OFF + ((NK1 - 1) % RING) * STAGE);"
    assert wm in src
    out["F"] = src.replace(wm, "reinterpret_cast<float*>(lds + RING_OFF + 2 * STAGE + 4096);")
    dma = """      bl_lds16(buf_rsrc(arr ? p.bi[2] : p.sc[2], CIO * 4), lds + SB3_OFF + (arr * CIO + pc * 256) * 4,
               (unsigned)(pc * 1024 + lane * 16), 0);"""
    assert dma in src, "dma"
    out["G"] = src.replace(dma, """      const float* srcp = (arr ? p.bi[2] : p.sc[2]) + pc * 256 + lane * 4;
      *reinterpret_cast<f4*>(lds + SB3_OFF + (arr * CIO + pc * 256) * 4 + lane * 16) = *reinterpret_cast<const f4*>(srcp);""")
    rd = """      const float* const sb3 = reinterpret_cast<const float*>(lds + SB3_OFF);
      const f4 s = *reinterpret_cast<const f4*>(sb3 + c0), b = *reinterpret_cast<const f4*>(sb3 + CIO + c0);"""
    assert rd in src, "rd"
    out["J"] = src.replace(rd, """      const f4 s = *reinterpret_cast<const f4*>(p.sc[2] + c0), b = *reinterpret_cast<const f4*>(p.bi[2] + c0);""")
    out["K"] = src.replace(rd, """      const float* const sb3 = reinterpret_cast<const float*>(lds + SB3_OFF);
      const f4 s = *reinterpret_cast<const f4*>(sb3 + c0), b = *reinterpret_cast<const f4*>(p.bi[2] + c0);""")
    out["L"] = src.replace(rd, """      const float* const sb3 = reinterpret_cast<const float*>(lds + SB3_OFF);
      const f4 s = *reinterpret_cast<const f4*>(p.sc[2] + c0), b = *reinterpret_cast<const f4*>(sb3 + CIO + c0);""")
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    src = subprocess.run(["git", "-C", ROOT, "show", "8308d2f:person-recognition-for-pose-estimation_amd/csrc/conv_bneck.hip"],
                         capture_output=True, text=True, check=True).stdout
    others = [o for o in glob.glob(os.path.join(BUILD, "*.o")) if not o.endswith("conv_bneck.o")]
    for k, s in variants(src).items():
        tmp = os.path.join(OUT, f"conv_bneck_8308{k}.hip")
        open(tmp, "w").write(s)
        obj = tmp[:-4] + ".o"
        r = subprocess.run([HIPCC, *FLAGS, "-c", tmp, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            sys.exit(f"variant {k}: {r.stderr[-3000:]}")
        lib = os.path.join(OUT, f"libprpe_8308{k}.so")
        r = subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *others, obj, "-o", lib],
                           capture_output=True, text=True)
        if r.returncode:
            sys.exit(f"link {k}: {r.stderr[-2000:]}")
        os.remove(obj)
        print("built", os.path.relpath(lib, ROOT), flush=True)


if __name__ == "__main__":
    main()
