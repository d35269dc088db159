"""Static checks (container, no GPU) of the hand-synchronised kernels' gfx950 assembly.

The kernels stage operands into LDS by LDS-DMA (``buffer_load ... lds``) and protect each ring
stage with a hand-counted ``s_waitcnt vmcnt(N)`` + ``s_barrier`` (``wait_barrier<N>``, conv.h):
the count N says how many of the wave's most recent vector-memory operations may still be in
flight when the stage is read, i.e. it assumes the ORDER in which the source issues them. Two
compiler reorderings broke that assumption in round 3 and both are checked here,
on the control-flow graph of every kernel (loop back-edges included):

1. Hoisted LDS reads: a ``ds_read`` whose result is consumed after a raw (inline-asm)
   ``s_barrier`` on some path -- the machine scheduler moved a read of the next stage above the barrier that
   publishes it (the run-to-run race at bs=256). The walk follows branches and loop back-edges,
   so a read scheduled into a loop tail and consumed after the loop-top barrier of the next
   iteration is found too.
2. Issue order under a counted wait: for every ``s_waitcnt vmcnt(N)`` with N > 0 written in
   inline asm (the hand-counted ones; the compiler's own waits are exact by construction), walk
   back along every CFG path over the N + 1 youngest vector-memory operations. The N-th is the
   oldest one the wait leaves in flight, the (N + 1)-th the youngest it must cover. If both lie
   in one scheduling region (a basic block between ``sched_barrier(0)`` fences / EXEC writes:
   where the machine scheduler may reorder) and that region holds both LDS-DMA and other
   vector-memory operations, whether the count covers the DMA pieces of the stage about to be
   read is the scheduler's choice, not the source's: an ORDER VIOLATION (the balanced-map build
   whose A loads were hoisted above the W pieces, max error 0.1). The fix is a
   ``__builtin_amdgcn_sched_barrier(0)`` between the DMA issue and the other accesses, as in
   conv_bneck.hip. (LDS-DMA pieces of one region are not reordered among themselves: each writes
   LDS through M0 at an address the compiler cannot separate from the others'. Ops the compiler
   ADDS -- scratch spills -- only make a count more conservative: a perf lint, below.)

3. Store data overwritten too early (round 5): a buffer / global store of more
   than 64 bits whose data VGPRs a VALU or MFMA writes within ``STORE_DATA_STATES`` wait states
   after it, on some CFG path. LLVM's hazard recognizer skips this for buffer stores with an SGPR
   soffset; on gfx950 it corrupts the stored data (the reverted commit 8308d2f: nine such stores,
   layer1 garbage; the same stream with ``s_nop 1`` after each store passed, with it before each
   store failed, tools/bneck_8308_nop.py). The source-level fix is conv_bneck.hip's
   ``store_data_guard``.

Perf lints (``--lint``, informational): compiler waits that drain a just-issued store (a load
issued behind a store: the round-3 bottleneck epilogue), and scratch accesses in kernels with
counted waits.

    python tools/barrier_hoist_check.py [--verbose] person-recognition-for-pose-estimation_amd/csrc/*.hip
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REG = re.compile(r"\b([vas])\[(\d+):(\d+)\]|\b([vas])(\d+)\b")
BRANCH = re.compile(r"^s_(c)?branch\w*\s+(\.LBB\w+)")
STORE_PREFIX = ("ds_write", "ds_store", "buffer_store", "global_store", "scratch_store", "flat_store")
VMEM_PREFIX = ("buffer_", "global_", "scratch_", "flat_", "tbuffer_")
VMEM_NOT_COUNTED = ("buffer_inv", "buffer_wbl2", "buffer_wbinvl1", "buffer_gl")
# wait states a >64-bit store's data VGPRs must stay unwritten: 2, the fix verified on the GPU
# (``s_nop 1`` after each store, tools/bneck_8308_nop.py) and LLVM's gfx940+ VMEM-store-data
# hazard model (2 VALU wait states); one state is unverified and not taken as safe
STORE_DATA_STATES = 2


def regs(txt):
    out = set()
    for m in REG.finditer(txt):
        if m.group(1):
            out |= {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


class Inst:
    __slots__ = ("idx", "text", "mn", "ops", "asm", "region", "block", "line")

    def __init__(self, idx, text, asm, line):
        self.idx, self.text, self.asm, self.line = idx, text, asm, line
        p = text.split(None, 1)
        self.mn = p[0]
        self.ops = p[1] if len(p) > 1 else ""
        self.region = self.block = -1

    @property
    def is_dma(self):
        return self.mn.startswith(("buffer_load", "global_load")) and (
            re.search(r"\blds\b", self.ops) is not None or "_lds_" in self.mn)

    @property
    def is_vmem(self):
        return self.mn.startswith(VMEM_PREFIX) and not self.mn.startswith(VMEM_NOT_COUNTED)

    @property
    def is_lds_read(self):
        return self.mn.startswith(("ds_read", "ds_load"))

    def dst(self):
        return regs(self.ops.split(",")[0])

    def srcs(self):
        if self.mn.startswith(STORE_PREFIX) or self.mn.startswith("s_waitcnt"):
            return regs(self.ops) if not self.mn.startswith("s_waitcnt") else set()
        return regs(",".join(self.ops.split(",")[1:]))

    def writes(self):
        if self.mn.startswith(STORE_PREFIX) or self.mn.startswith(("s_waitcnt", "s_barrier", "s_nop")):
            return set()
        return self.dst()


class Kernel:
    """One function of the .s: instructions, basic blocks, CFG, scheduling regions."""

    def __init__(self, name, lines, first_line=0):
        self.name = name
        insts, starts = [], [0]
        lab_pos, pending = {}, []                      # label -> index of the next instruction
        in_asm = False
        ended = False                                  # the previous instruction ends its block
        for ln, raw in enumerate(lines):
            s = raw.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            m = re.match(r"^(\.LBB\w+):", s)
            if m or s.startswith("; %bb."):
                starts.append(len(insts))
                if m:
                    pending.append(m.group(1))
                ended = False
                continue
            if s.startswith("; sched_barrier mask(0x00000000)"):
                code = "FENCE"
            else:
                code = s.split(";")[0].strip()
                if not code or code.startswith(".") or code.endswith(":"):
                    continue
            if ended:
                starts.append(len(insts))
                ended = False
            for l in pending:
                lab_pos[l] = len(insts)
            pending = []
            insts.append(Inst(len(insts), code, in_asm, first_line + ln + 1))
            if BRANCH.match(code) or code.startswith(("s_endpgm", "s_setpc")):
                ended = True
        for l in pending:
            lab_pos[l] = len(insts)
        self.insts = insts
        starts = sorted(set(x for x in starts if x < len(insts)))
        self.blocks = list(zip(starts, starts[1:] + [len(insts)]))
        bstart = {a: i for i, (a, _) in enumerate(self.blocks)}
        self.succ = [[] for _ in self.blocks]
        blk_of = {}
        for bi, (a, b) in enumerate(self.blocks):
            for i in range(a, b):
                insts[i].block = bi
                blk_of[i] = bi
        for bi, (a, b) in enumerate(self.blocks):
            last = insts[b - 1]
            m = BRANCH.match(last.text)
            nxt = bi + 1 if bi + 1 < len(self.blocks) else None
            if last.mn.startswith(("s_endpgm", "s_setpc")):
                continue
            if m:
                tgt = lab_pos.get(m.group(2))
                if tgt is None or tgt not in bstart:
                    raise ValueError(f"{name}: branch target {m.group(2)} is not a block start")
                self.succ[bi].append(bstart[tgt])
                if m.group(1) and nxt is not None:
                    self.succ[bi].append(nxt)
            elif nxt is not None:
                self.succ[bi].append(nxt)
        self.pred = [[] for _ in self.blocks]
        for bi, ss in enumerate(self.succ):
            for s_ in ss:
                self.pred[s_].append(bi)
        # scheduling regions: split blocks at fences and EXEC writes
        r = -1
        for bi, (a, b) in enumerate(self.blocks):
            r += 1
            for i in range(a, b):
                it = insts[i]
                if it.text == "FENCE" or re.match(r"^\S+\s+exec\b", it.text):
                    r += 1
                    it.region = -1
                    continue
                it.region = r
        self.region_kinds = {}
        for it in insts:
            if it.region >= 0 and it.is_vmem:
                k = self.region_kinds.setdefault(it.region, set())
                k.add("dma" if it.is_dma else "vmem")

    # ---- check 1: LDS reads hoisted above a barrier
    def hoisted_reads(self):
        bad = []
        for it in self.insts:
            # LDS reads written as inline asm are placed by the source, not by the scheduler (a
            # volatile asm keeps its order against the barrier asm): they cannot be hoisted, and
            # their results may legitimately live across later barriers (the upconv's H rows)
            if not it.is_lds_read or it.asm:
                continue
            dst = it.dst()
            if not dst:
                continue
            if self._reaches_barrier_before_use(it, dst):
                bad.append(it)
        return bad

    def _reaches_barrier_before_use(self, it, dst):
        """Is the read's value consumed after an inline-asm s_barrier on some path (before being
        overwritten)? Only raw barriers (wait_barrier, conv.h) are invisible to the compiler's
        memory model; __syncthreads() is a workgroup fence it does not move LDS reads across, so a
        read before one of those is the source's own. A path that passes a barrier and never uses
        the value (dead there, e.g. an exec-skipped use) is not a hazard."""
        stack = [(it.block, it.idx + 1, False)]
        seen = set()
        while stack:
            bi, start, crossed = stack.pop()
            _, b = self.blocks[bi]
            done = False
            for i in range(start, b):
                x = self.insts[i]
                if x.mn.startswith("s_barrier") and x.asm:
                    crossed = True
                    continue
                if dst & x.srcs():
                    if crossed:
                        return True
                    done = True
                    break
                if dst & x.writes():
                    done = True
                    break
            if done:
                continue
            for s_ in self.succ[bi]:
                if (s_, crossed) not in seen:
                    seen.add((s_, crossed))
                    stack.append((s_, self.blocks[s_][0], crossed))
        return False

    # ---- check 2: counted vmcnt waits vs scheduling regions
    def counted_waits(self):
        out = []
        for it in self.insts:
            if it.asm and it.mn == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", it.ops)
                if m and int(m.group(1)) > 0:
                    out.append((it, int(m.group(1))))
        return out

    def windows(self, it, n, cap=4096):
        """Every distinct sequence of the n + 1 youngest vector-memory ops before ``it`` along a
        CFG path (shorter where the kernel entry is reached first)."""
        res = set()
        stack = [(it.block, it.idx, ())]
        seen = {}
        while stack and len(res) < cap:
            bi, end, seq = stack.pop()
            a, _ = self.blocks[bi]
            for i in range(end - 1, a - 1, -1):
                x = self.insts[i]
                if x.is_vmem:
                    seq = seq + (x.idx,)
                    if len(seq) == n + 1:
                        break
            if len(seq) == n + 1 or not self.pred[bi]:
                res.add(seq)
                continue
            for p in self.pred[bi]:
                key = (p, seq)
                if seen.get(key):
                    continue
                seen[key] = True
                stack.append((p, self.blocks[p][1], seq))
        return res

    def order_violations(self):
        waits = self.counted_waits()
        viol, nwin = [], 0
        for w, n in waits:
            for seq in self.windows(w, n):
                nwin += 1
                if len(seq) <= n:
                    continue
                o_n, o_n1 = self.insts[seq[n - 1]], self.insts[seq[n]]
                if o_n.region == o_n1.region and o_n.region >= 0 and self.region_kinds.get(o_n.region) == {"dma", "vmem"}:
                    viol.append((w, n, seq, "window boundary inside a region mixing LDS-DMA and other vector-memory ops"))
        return waits, nwin, viol


    # ---- check 3: store data overwritten inside the store's data-read window
    def store_data_overwrites(self, states=STORE_DATA_STATES):
        """A buffer / global store of more than 64 bits reads its data VGPRs some cycles after
        it issues; a VALU write of those VGPRs fewer than ``states`` wait states later (an
        ``s_nop N`` counts N + 1, any other instruction 1; followed along every CFG path) can
        replace the data before it is read.  LLVM models this hazard only for stores whose
        soffset is not an SGPR, so the compiler emits it freely for ``buffer_store ... sN offen``.
        On gfx950 it is real: the reverted commit 8308d2f's identity-block epilogue had nine such
        stores and wrote garbage; two wait states after each (tools/bneck_8308_nop.py) fixed it."""
        out = []
        for it in self.insts:
            if not it.mn.startswith(("buffer_store_dwordx3", "buffer_store_dwordx4", "global_store_dwordx3",
                                     "global_store_dwordx4", "flat_store_dwordx3", "flat_store_dwordx4")):
                continue
            ops = [o.strip() for o in it.ops.split(",")]
            data = regs(ops[1] if it.mn.startswith(("global_", "flat_")) else ops[0])
            stack, hit = [(it.block, it.idx + 1, 0)], None
            seen = set()
            while stack and hit is None:
                bi, start, ws = stack.pop()
                _, b = self.blocks[bi]
                for i in range(start, b):
                    if ws >= states:
                        break
                    x = self.insts[i]
                    if x.text == "FENCE":
                        continue
                    if x.mn.startswith("v_") and data & x.writes():
                        hit = x
                        break
                    m = re.match(r"s_nop\s+(\d+)", x.text)
                    ws += int(m.group(1)) + 1 if m else 1
                else:
                    for s_ in self.succ[bi]:
                        if (s_, ws) not in seen:
                            seen.add((s_, ws))
                            stack.append((s_, self.blocks[s_][0], ws))
            if hit is not None:
                out.append((it, hit))
        return out


def store_drains(k):
    """Perf lint: compiler-inserted ``s_waitcnt vmcnt(N)`` for a load issued right after a STORE
    (a store among the three youngest ops the wait must complete, on some path): one in-order
    counter for loads, stores and LDS-DMA, so the wait exposes that store's latency too."""
    out = []
    for it in k.insts:
        if it.asm or it.mn != "s_waitcnt":
            continue
        m = re.search(r"vmcnt\((\d+)\)", it.ops)
        if not m:
            continue
        n = int(m.group(1))
        for seq in k.windows(it, n + 2, cap=64):
            if any(k.insts[i].mn.startswith(("buffer_store", "global_store")) for i in seq[n:n + 3]):
                out.append(it)
                break
    return out


def kernels_of(asm_lines):
    starts = [i for i, l in enumerate(asm_lines) if re.match(r"^_Z\w+:", l)]
    out = []
    for a in starts:
        b = next((j for j in range(a, len(asm_lines)) if asm_lines[j].startswith(".Lfunc_end")), len(asm_lines))
        out.append(Kernel(asm_lines[a].split(":")[0], asm_lines[a + 1:b], a + 1))
    return out


def compile_asm(src, out):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                    "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "person-recognition-for-pose-estimation_amd", "csrc"),
                    "--cuda-device-only", "-S", "-o", out, src], check=True, capture_output=True)


def check_asm(path, verbose=False, label=None, lint=False):
    """-> (hoisted ds_reads, order violations, counted waits, windows, store-data overwrites)
    summed over the kernels."""
    lines = open(path).read().split("\n")
    label = label or os.path.basename(path)
    nh = nv = nw = nwin = ns = 0
    for k in kernels_of(lines):
        h = k.hoisted_reads()
        waits, nwin_k, v = k.order_violations()
        sd = k.store_data_overwrites()
        ns += len(sd)
        if sd:
            print(f"{label} {k.name[:90]}: {len(sd)} store(s) whose data VGPRs the next instruction overwrites")
            for st, x in sd[:4]:
                print("    ", st.line, st.text, "|", x.text)
        nh += len(h)
        nv += len(v)
        nw += len(waits)
        nwin += nwin_k
        if h:
            print(f"{label} {k.name[:90]}: {len(h)} ds_read(s) hoisted above an s_barrier")
            for it in h[:4]:
                print("    ", it.line, it.text)
        if v:
            print(f"{label} {k.name[:90]}: {len(v)} issue-order violation(s) under counted waits")
            for w, n, seq, why in v[:4]:
                where = f"vmcnt({n}) at asm line {w.line}" if w else "kernel"
                print(f"     {where}: {why}; ops " + ", ".join(k.insts[i].text[:48] for i in seq[max(0, n - 2):n + 1]))
        if lint and k.counted_waits() and any(x.mn.startswith("scratch_") for x in k.insts):
            print(f"{label} {k.name[:90]}: lint: scratch accesses (a private array or spill) in a kernel "
                  f"with counted waits")
        if lint:
            d = store_drains(k)
            if d:
                print(f"{label} {k.name[:90]}: lint: {len(d)} compiler vmcnt wait(s) draining a store "
                      f"(asm lines {', '.join(str(x.line) for x in d[:6])})")
        if verbose and waits:
            print(f"{label} {k.name[:90]}: {len(waits)} counted wait(s), {nwin_k} issue-order window(s) checked")
    return nh, nv, nw, nwin, ns


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("srcs", nargs="+")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--lint", action="store_true", help="also list compiler waits that drain a store")
    a = ap.parse_args()
    tot = [0, 0, 0, 0, 0]
    for src in a.srcs:
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "k.s")
            if src.endswith(".s"):
                out = src
            else:
                compile_asm(src, out)
            r = check_asm(out, a.verbose, os.path.basename(src), a.lint)
        tot = [x + y for x, y in zip(tot, r)]
    print(f"counted vmcnt waits: {tot[2]}, issue-order windows checked: {tot[3]}")
    print("total hoisted ds_reads:", tot[0])
    print("total issue-order violations:", tot[1])
    print("total store-data overwrites:", tot[4])
    return 1 if tot[0] or tot[1] or tot[4] else 0


if __name__ == "__main__":
    sys.exit(main())
