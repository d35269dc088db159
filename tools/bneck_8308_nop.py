"""Round-5 causal test for the reverted commit 8308d2f (container side; measurement only, nothing
here ships). tools/barrier_hoist_check.py (check 3) finds, in every failing 8308d2f variant (A-G of
tools/bneck_8308_variants.py) and in none of the passing ones (J, K, L, the parent commit, HEAD),
128-bit buffer stores of the identity-block epilogue whose data VGPRs the very next VALU
instruction overwrites.  This script rebuilds variant A with its device assembly patched, so that
the instruction stream is otherwise the one that fails:

  N  A + `s_nop 1` AFTER each such store (two wait states between the store and the overwrite)
  P  A + `s_nop 1` BEFORE each such store (the same added cycles, the overwrite still adjacent;
     the control)

and links each with the current build's other objects into tools/abl/libprpe_8308<X>.so for
tools/bneck_8308.sh.  The hipcc pipeline is taken from `hipcc -### -save-temps`: the device
steps up to the .s run as hipcc would, the .s is patched, the rest (assembler, lld, bundler, host
compile) runs unchanged.

    python tools/bneck_8308_nop.py [N P]
"""
import glob
import importlib.util
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")
BUILD = os.path.join(PKG, "build")
OUT = os.path.join(ROOT, "tools", "abl")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "include"),
         "-I" + os.path.join(PKG, "csrc"), "-Wno-unused-result"]


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def patch(asm, where):
    """Insert `s_nop 1` before or after every store the hazard scan flags; returns (text, count)."""
    chk = _load("barrier_hoist_check")
    lines = asm.split("\n")
    sites = {st.line - 1 for k in chk.kernels_of(lines) for st, _ in k.store_data_overwrites()}
    out = []
    for i, l in enumerate(lines):
        if i in sites and where == "before":
            out.append("\ts_nop 1")
        out.append(l)
        if i in sites and where == "after":
            out.append("\ts_nop 1")
    return "\n".join(out), len(sites)


def build(tag, src, where, others):
    work = os.path.join(OUT, "st_" + tag)
    os.makedirs(work, exist_ok=True)
    hip = os.path.join(work, f"v{tag}.hip")
    open(hip, "w").write(src)
    obj = os.path.join(work, f"v{tag}.o")
    r = subprocess.run([HIPCC, "-###", *FLAGS, "-save-temps", "-c", hip, "-o", obj], cwd=work,
                       capture_output=True, text=True)
    cmds = [l for l in r.stderr.splitlines() if l.startswith(' "')]
    dev_s = f"v{tag}-hip-amdgcn-amd-amdhsa-gfx950.s"
    k = next(i for i, c in enumerate(cmds) if f'"-o" "{dev_s}"' in c)
    for c in cmds[:k + 1]:
        subprocess.run(shlex.split(c), cwd=work, check=True, capture_output=True)
    path = os.path.join(work, dev_s)
    text, n = patch(open(path).read(), where)
    assert n > 0, "no flagged store in variant A"
    open(path, "w").write(text)
    for c in cmds[k + 1:]:
        subprocess.run(shlex.split(c), cwd=work, check=True, capture_output=True)
    lib = os.path.join(OUT, f"libprpe_8308{tag}.so")
    subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *others, obj, "-o", lib], check=True,
                   capture_output=True)
    print(f"built {os.path.relpath(lib, ROOT)} ({n} stores patched, s_nop {where})", flush=True)


def main():
    want = sys.argv[1:] or ["N", "P"]
    os.makedirs(OUT, exist_ok=True)
    others = [o for o in glob.glob(os.path.join(BUILD, "*.o")) if not o.endswith("conv_bneck.o")]
    assert any(o.endswith("build_info.o") for o in others), "run build.py first"
    src = subprocess.run(["git", "-C", ROOT, "show",
                          "8308d2f:person-recognition-for-pose-estimation_amd/csrc/conv_bneck.hip"],
                         capture_output=True, text=True, check=True).stdout
    a = _load("bneck_8308_variants").variants(src)["A"]
    for tag in want:
        build(tag, a, {"N": "after", "P": "before"}[tag], others)


if __name__ == "__main__":
    main()
