"""Build a phase-timestamp variant of the fused bottleneck (container; measurement only): a
scratch copy of csrc/conv_bneck.hip in which wave 0 of every workgroup records the device's
constant 100-MHz clock (s_memrealtime) at its phase boundaries plus the hardware slot it ran on
(HW_ID, XCC_ID), into a device array read back by an extra export, prpe_bneck_trace_read.
Linked with the current build's other objects and build_info.o (same source hash) as
tools/abl/libprpe_trace.so; tools/bneck_trace.py loads it on the box.

Question it answers (kernel 5.21 ms ~ skeleton 3.11 + MFMA phases): how long
each phase of one tile takes, and whether the two workgroups sharing a CU overlap their
memory phases (1 and 3) with each other's MFMA phase (2) or run them in step.

    python tools/bneck_trace_build.py
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
SLOTS = 64         # u64 per workgroup: T0 start, T1 phase-1 K-loop done, T1b t1 in LDS, T2 phase-2
                   # K-loop done, T2b t2 in LDS, T3 end, HW_ID, XCC_ID; then per phase-1 K-step kt
                   # (low 32 bits): slot 8 + kt past its wait + barrier, slot 8 + NK1 + kt past the
                   # split of A(kt) (its loads landed), slot 8 + 2 NK1 + kt past its MFMAs' issue
MAXWG = 1 << 17

EDITS = [
    ("namespace prpe_k {\n\nstruct BneckK {",
     f"namespace prpe_k {{\n__device__ unsigned long long bneck_trace_buf[{SLOTS} * {MAXWG}];\n\nstruct BneckK {{"),
    ("  const int oh0 = th * TR, ow0 = tw * TC;\n",
     "  const int oh0 = th * TR, ow0 = tw * TC;\n  const unsigned long long T0 = __builtin_amdgcn_s_memrealtime();\n"),
    ("#pragma unroll\n  for (int kt = 0; kt < NK1; ++kt) {\n    const int m = na_step(kt);",
     "  unsigned TS[NK1], TSS[NK1], TM[NK1];\n#pragma unroll\n  for (int kt = 0; kt < NK1; ++kt) {\n    const int m = na_step(kt);"),
    ("      else wait_barrier<2 * PPW>();\n    }\n    issue_wu(kt + RING - 1);",
     "      else wait_barrier<2 * PPW>();\n    }\n    TS[kt] = (unsigned)__builtin_amdgcn_s_memrealtime();\n    issue_wu(kt + RING - 1);"),
    ("    split(kt);\n    if (kt + AD < NK1) load_a(kt + AD);",
     "    split(kt);\n    asm volatile(\"\" :: \"v\"(af[0][0]), \"v\"(af[0][1]), \"v\"(af[1][0]));\n"
     "    TSS[kt] = (unsigned)__builtin_amdgcn_s_memrealtime();\n    if (kt + AD < NK1) load_a(kt + AD);"),
    ("      if (two) acc1[1][j] = mfma3t(b, af[1], acc1[1][j]);\n    }\n  }\n",
     "      if (two) acc1[1][j] = mfma3t(b, af[1], acc1[1][j]);\n    }\n"
     "    asm volatile(\"\" :: \"v\"(acc1[0][NJ1 - 1]), \"v\"(acc1[1][NJ1 - 1]));\n"
     "    TM[kt] = (unsigned)__builtin_amdgcn_s_memrealtime();\n  }\n"),
    ("  // epilogue 1: bn1 + ReLU", "  const unsigned long long T1 = __builtin_amdgcn_s_memrealtime();\n  // epilogue 1: bn1 + ReLU"),
    ("  // =========================== phase 2: t2 = conv2(t1)",
     "  const unsigned long long T1b = __builtin_amdgcn_s_memrealtime();\n  // =========================== phase 2: t2 = conv2(t1)"),
    ("  // epilogue 2: bn2 + ReLU", "  const unsigned long long T2 = __builtin_amdgcn_s_memrealtime();\n  // epilogue 2: bn2 + ReLU"),
    ("  // =========================== phase 3: y",
     "  const unsigned long long T2b = __builtin_amdgcn_s_memrealtime();\n  // =========================== phase 3: y"),
    ("  if (!ovq) ymax = 0.f;                                      // (an invalid pixel's y is relu(bias))\n",
     "  if (!ovq) ymax = 0.f;                                      // (an invalid pixel's y is relu(bias))\n"
     "  {\n    const unsigned long long T3 = __builtin_amdgcn_s_memrealtime();\n"
     "    unsigned hw, xcc;\n"
     "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(hw));\n"
     "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc));\n"
     f"    if (tid == 0 && blockIdx.x < {MAXWG}) {{\n"
     f"      unsigned long long* o = bneck_trace_buf + (size_t)blockIdx.x * {SLOTS};\n"
     "      o[0] = T0; o[1] = T1; o[2] = T1b; o[3] = T2; o[4] = T2b; o[5] = T3; o[6] = hw; o[7] = xcc;\n"
     "      for (int k = 0; k < NK1; ++k) { o[8 + k] = TS[k]; o[8 + NK1 + k] = TSS[k]; o[8 + 2 * NK1 + k] = TM[k]; }\n"
     "    }\n  }\n"),
]
TAIL = f"""
extern "C" int prpe_bneck_trace_read(void* dst, unsigned long long bytes) {{
  if (bytes > sizeof(unsigned long long) * {SLOTS} * {MAXWG}) return -22;
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(prpe_k::bneck_trace_buf), bytes, 0, hipMemcpyDeviceToHost);
}}
"""


def main():
    os.makedirs(OUT, exist_ok=True)
    others = [o for o in glob.glob(os.path.join(BUILD, "*.o")) if not o.endswith("conv_bneck.o")]
    assert any(o.endswith("build_info.o") for o in others), "run build.py first"
    s = open(os.path.join(CSRC, "conv_bneck.hip")).read()
    for a, b in EDITS:
        assert s.count(a) == 1, a
        s = s.replace(a, b)
    s += TAIL
    tmp = os.path.join(OUT, "conv_bneck_trace.hip")
    open(tmp, "w").write(s)
    obj = tmp[:-4] + ".o"
    r = subprocess.run([HIPCC, *FLAGS, "-c", tmp, "-o", obj], capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    lib = os.path.join(OUT, "libprpe_trace.so")
    r = subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *others, obj, "-o", lib],
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    os.remove(obj)
    print("built", os.path.relpath(lib, ROOT))


if __name__ == "__main__":
    main()
