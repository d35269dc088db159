"""Static check (container, no GPU): LDS reads the compiler scheduled ABOVE a workgroup barrier.

A K-loop step reads its LDS stage only after ``wait_barrier`` (s_waitcnt vmcnt(N) + s_barrier:
every wave's LDS-DMA pieces of that stage have landed). If the machine scheduler hoists a
ds_read of the next step above that s_barrier, the read can see a stage another wave's DMA has
not finished writing: a data race that shows as run-to-run differences at large grids. For every
kernel of a HIP source this prints the ds_reads whose destination registers are not used before
the next s_barrier (i.e. they feed only work after it).

    python tools/barrier_hoist_check.py person-recognition-for-pose-estimation_amd/csrc/*.hip
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REG = re.compile(r"\b([vas])\[(\d+):(\d+)\]|\b([vas])(\d+)\b")


def regs(txt):
    out = set()
    for m in REG.finditer(txt):
        if m.group(1):
            out |= {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def check(asm_lines):
    starts = [i for i, l in enumerate(asm_lines) if re.match(r"^_Z\w+:", l)] + [len(asm_lines)]
    bad = {}
    for a, b in zip(starts, starts[1:]):
        name = asm_lines[a].split(":")[0]
        body = [l.split(";")[0].strip() for l in asm_lines[a:b]]
        bars = [i for i, s in enumerate(body) if s.startswith("s_barrier")]
        for i, s in enumerate(body):
            if not (s.startswith("ds_read") or s.startswith("ds_load")):
                continue
            nb = next((j for j in bars if j > i), None)
            if nb is None:
                continue
            parts = s.split(None, 1)
            if len(parts) < 2:
                continue
            dst = regs(parts[1].split(",")[0])
            used = False
            for s2 in body[i + 1:nb]:
                p2 = s2.split(None, 1)
                if len(p2) < 2 or p2[0].startswith("s_waitcnt"):
                    continue
                ops = p2[1].split(",")
                srcs = regs(",".join(ops[1:])) if not p2[0].startswith(("ds_write", "buffer_store", "global_store")) \
                    else regs(p2[1])
                if dst & srcs:
                    used = True
                    break
                if dst & regs(ops[0]) and not p2[0].startswith(("ds_write", "buffer_store", "global_store")):
                    break                                   # overwritten before any use
            if not used:
                bad.setdefault(name, []).append((i, s))
    return bad


def main():
    nbad = 0
    for src in sys.argv[1:]:
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "k.s")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                            "-I" + os.path.join(ROOT, "include"),
                            "-I" + os.path.join(ROOT, "person-recognition-for-pose-estimation_amd", "csrc"),
                            "--cuda-device-only", "-S", "-o", out, src], check=True, capture_output=True)
            lines = open(out).read().split("\n")
        for name, items in check(lines).items():
            nbad += len(items)
            print(f"{os.path.basename(src)} {name[:90]}: {len(items)} ds_read(s) hoisted above an s_barrier")
            for i, s in items[:4]:
                print("    ", i, s)
    print("total hoisted ds_reads:", nbad)
    return 1 if nbad else 0


if __name__ == "__main__":
    sys.exit(main())
