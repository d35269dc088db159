"""CPU (no GPU): static checks of the gfx950 assembly of every HIP source
(tools/barrier_hoist_check.py), over each kernel's control-flow graph:

* no LDS read consumed after a raw (inline-asm) ``s_barrier`` it was scheduled above -- the
  round-3 race that made fused-bottleneck frames differ between runs at bs=256;
  the walk follows loop back-edges, so a read moved into a loop tail is seen against the
  loop-top barrier of the next iteration;
* no hand-counted ``s_waitcnt vmcnt(N)`` whose window boundary (the N-th / (N+1)-th youngest
  vector-memory op on some path) falls inside a scheduling region that mixes LDS-DMA with other
  vector-memory ops -- where the scheduler, not the source, decides whether the count covers the
  DMA pieces of the stage about to be read (the round-3 balanced-map build, max error 0.1);
* no 128-bit store whose data VGPRs the very next instruction overwrites -- the gfx950
  store-data hazard LLVM does not model for SGPR-offset buffer stores, the cause of the reverted
  commit 8308d2f's garbage layer1 blocks: the check flags that commit's
  conv_bneck.hip and passes HEAD's.

The synthetic cases pin the checker's own logic; the real test compiles all csrc/*.hip in
parallel (hipcc --cuda-device-only -S; the largest sources take 2-3 minutes). Skipped without
hipcc."""
import concurrent.futures as cf
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "person-recognition-for-pose-estimation_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import barrier_hoist_check as B  # noqa: E402

HIPCC = os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("hipcc")


def _kernel(body):
    return B.Kernel("_Zk", body.strip("\n").split("\n"))


def test_checker_follows_loop_back_edges_for_hoisted_reads():
    # the ds_read in the loop tail feeds the MFMA after the NEXT iteration's raw barrier
    k = _kernel("""
\ts_mov_b32 s0, 0
.LBB0_1:
;;#ASMSTART
\ts_waitcnt vmcnt(0)
\ts_barrier
;;#ASMEND
\tv_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], v[0:3]
\tds_read_b128 v[8:11], v20
\ts_add_u32 s0, s0, 1
\ts_cmp_lg_u32 s0, 8
\ts_cbranch_scc1 .LBB0_1
\ts_endpgm
""")
    assert len(k.hoisted_reads()) == 1
    # the same read consumed before the barrier: fine
    k = _kernel("""
.LBB0_1:
;;#ASMSTART
\ts_barrier
;;#ASMEND
\tds_read_b128 v[8:11], v20
\tv_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], v[0:3]
\ts_cbranch_scc1 .LBB0_1
\ts_endpgm
""")
    assert k.hoisted_reads() == []


def test_checker_flags_a_count_whose_boundary_splits_a_mixed_region():
    # vmcnt(2) must cover the DMA piece; the two register loads after it may stay in flight.
    fenced = """
\tbuffer_load_dwordx4 v2, s[4:7], 0 offen lds
\t; sched_barrier mask(0x00000000)
\tbuffer_load_dwordx4 v[10:13], v18, s[8:11], 0 offen
\tbuffer_load_dwordx4 v[14:17], v18, s[8:11], 0 offen offset:16
;;#ASMSTART
\ts_waitcnt vmcnt(2)
\ts_barrier
;;#ASMEND
\ts_endpgm
"""
    waits, nwin, viol = _kernel(fenced).order_violations()
    assert len(waits) == 1 and nwin == 1 and viol == []
    # no fence: DMA and loads share one region, the count's boundary falls between them
    waits, nwin, viol = _kernel(fenced.replace("\t; sched_barrier mask(0x00000000)\n", "")).order_violations()
    assert len(viol) == 1
    # the window reaching back through both arms of a branch: every path is checked
    k = _kernel("""
\tbuffer_load_dwordx4 v2, s[4:7], 0 offen lds
\tbuffer_load_dwordx4 v[10:13], v18, s[8:11], 0 offen
\ts_cbranch_vccnz .LBB0_2
; %bb.1:
\tbuffer_load_dwordx4 v[14:17], v18, s[8:11], 0 offen offset:16
.LBB0_2:
;;#ASMSTART
\ts_waitcnt vmcnt(1)
\ts_barrier
;;#ASMEND
\ts_endpgm
""")
    assert len(k.windows(k.counted_waits()[0][0], 1)) == 2 and len(k.order_violations()[2]) == 1


@pytest.fixture(scope="module")
def asm_dir():
    if not HIPCC:
        pytest.skip("no hipcc")
    td = tempfile.mkdtemp(prefix="prpe_isa_")
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))

    def one(src):
        out = os.path.join(td, os.path.basename(src)[:-4] + ".s")
        B.compile_asm(src, out)
        return out

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 8)) as ex:
        outs = list(ex.map(one, srcs))
    yield outs
    shutil.rmtree(td, ignore_errors=True)


def test_checker_flags_store_data_overwritten_by_the_next_instruction():
    body = """
\tbuffer_store_dwordx4 v[36:39], v81, s[12:15], s25 offen
\tv_pk_mul_f32 v[36:37], v[64:65], v[56:57]
\ts_endpgm
"""
    assert len(_kernel(body).store_data_overwrites()) == 1
    # one wait state (s_nop 0, or one unrelated instruction) is not enough: still flagged
    assert len(_kernel(body.replace("\tv_pk", "\ts_nop 0\n\tv_pk")).store_data_overwrites()) == 1
    assert len(_kernel(body.replace("\tv_pk", "\tv_add_u32_e32 v1, 4, v2\n\tv_pk")).store_data_overwrites()) == 1
    # two wait states (s_nop 1, the GPU-verified fix, or two unrelated instructions): clear
    assert _kernel(body.replace("\tv_pk", "\ts_nop 1\n\tv_pk")).store_data_overwrites() == []
    assert _kernel(body.replace("\tv_pk", "\tv_add_u32_e32 v1, 4, v2\n\ts_nop 0\n\tv_pk")).store_data_overwrites() == []
    assert _kernel(body.replace("\tv_pk", "\tv_add_u32_e32 v1, 4, v2\n\tv_add_u32_e32 v3, 4, v2\n\tv_pk"))\
        .store_data_overwrites() == []
    # 64-bit stores, and writes of other registers, are not flagged
    assert _kernel(body.replace("dwordx4 v[36:39]", "dwordx2 v[36:37]")).store_data_overwrites() == []
    assert _kernel(body.replace("v_pk_mul_f32 v[36:37]", "v_pk_mul_f32 v[40:41]")).store_data_overwrites() == []
    # an MFMA writing the data, and the overwrite in the next basic block: flagged
    assert len(_kernel(body.replace("v_pk_mul_f32 v[36:37], v[64:65], v[56:57]",
                                    "v_mfma_f32_16x16x32_f16 v[36:39], v[0:3], v[4:7], v[8:11]"))
               .store_data_overwrites()) == 1
    k = _kernel("""
\tglobal_store_dwordx4 v[0:1], v[36:39], off
.LBB0_2:
\tv_mov_b32_e32 v38, 0
\ts_endpgm
""")
    assert len(k.store_data_overwrites()) == 1


def test_store_data_check_fails_on_8308d2f_and_passes_head(asm_dir, tmp_path):
    r = subprocess.run(["git", "-C", ROOT, "show",
                        "8308d2f:person-recognition-for-pose-estimation_amd/csrc/conv_bneck.hip"],
                       capture_output=True, text=True)
    if r.returncode:
        pytest.skip("commit 8308d2f not in this checkout")
    src = tmp_path / "conv_bneck_8308d2f.hip"
    src.write_text(r.stdout)
    out = str(tmp_path / "k.s")
    B.compile_asm(str(src), out)
    bad = {k.name: len(k.store_data_overwrites()) for k in B.kernels_of(open(out).read().split("\n"))}
    ident = [n for n in bad if "Lb0E" in n]                 # the identity blocks (PROJ = false)
    assert ident and all(bad[n] > 0 for n in ident), bad    # the layer1 / layer2 blocks that failed
    head = [o for o in asm_dir if o.endswith("conv_bneck.s")][0]
    assert all(not k.store_data_overwrites() for k in B.kernels_of(open(head).read().split("\n")))


def test_every_kernel_source_has_no_hoisted_reads_and_no_order_violations(asm_dir, capsys):
    tot = [0, 0, 0, 0, 0]
    for out in asm_dir:
        r = B.check_asm(out)
        tot = [a + b for a, b in zip(tot, r)]
    text = capsys.readouterr().out
    print(text)
    hoisted, viol, waits, windows, stores = tot
    assert len(asm_dir) >= 13
    assert waits >= 100 and windows >= waits          # the hand-counted waits were found and walked
    assert hoisted == 0 and viol == 0 and stores == 0, text


def _kernel_meta(path):
    """kernel name -> (VGPRs, VGPR spills) from the .s metadata."""
    import re
    out = {}
    for blk in open(path).read().split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        out[name] = (int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1)),
                     int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1)))
    return out


def test_occupancy_critical_tiles_fit_128_vgprs_without_spills(asm_dir):
    # the precision-3 256x128 wave tile (the trunk's unfused convs) and the precision-4 4-wave
    # two-K-step tile (AdaFace) run two / four workgroups per CU only at <= 128 VGPRs; round 5's
    # GELU rewrite silently pushed them to 132 (one / three per CU: trunk convs 15-27 % slower).
    # Their launch bound now asks for 4 waves per SIMD; this pins that it costs no spills.
    #  every instantiation that conv_wave.hip's wave_wps maps to 4 waves per SIMD is
    # checked, not only the two measured ones: NW 8, TM 2, NP 2 without prologue (bf16, f16, dual,
    # planes-input variants alike) and NW 4, TM 2, single-plane (ONE) with KSF 1, no prologue
    meta = _kernel_meta([o for o in asm_dir if o.endswith("conv_wave.s")][0])

    def targs(name):   # NW, TM, TN, NP, STAGES, PRO, F16, DUAL, APL, ONE, KSF, X11 from the mangled name
        m = re.search(r"conv_wave_kernelI((?:L[ib]n?\d+E)+)E", name)
        return [int(v.replace("n", "-")) for v in re.findall(r"L[ib](n?\d+)E", m.group(1))] if m else None

    def wps4(a):
        nw, tm, _tn, np_, _st, pro, _f16, _dual, _apl, one, ksf, _x11 = a
        return (nw == 8 and tm == 2 and np_ == 2 and not pro) or (nw == 4 and tm == 2 and one and ksf == 1 and not pro)

    hot = {k: v for k, v in meta.items() if targs(k) and len(targs(k)) == 12 and wps4(targs(k))}
    # (the pixel-contiguous 1x1 forms, X11, included: same launch bound)
    assert any(targs(k)[11] for k in hot), sorted(hot)
    assert any("conv_wave_kernelILi8ELi2ELi8ELi2ELi3ELb0ELb1E" in k for k in hot), sorted(meta)   # p3 256x128
    assert any("conv_wave_kernelILi4ELi2ELi8ELi2ELi2ELb0ELb1ELb0ELb0ELb1ELi1E" in k for k in hot)   # p4, KSF 1
    assert len(hot) >= 4, sorted(hot)
    for k, (v, spill) in hot.items():
        assert v <= 128 and spill == 0, (k, v, spill)
