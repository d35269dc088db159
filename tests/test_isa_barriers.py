"""CPU (no GPU): the gfx950 assembly of the hand-synchronised fused kernels has no LDS read that
the compiler scheduled above a workgroup barrier (tools/barrier_hoist_check.py). Such a read
sees a ring stage before the other waves' LDS-DMA pieces of it have landed: the round-3 race
that made fused-bottleneck frames differ between runs at bs=256. Compiles each
source with hipcc --cuda-device-only -S (5-15 s each; conv_halo.hip and conv_wave.hip take 1.5-2
minutes and are checked by hand: 0 as well, round 3); skipped without hipcc."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "person-recognition-for-pose-estimation_amd", "csrc")


@pytest.mark.skipif(not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")), reason="no hipcc")
@pytest.mark.parametrize("src", ["conv_stem.hip", "conv_bneck.hip", "conv_gemm.hip", "attention.hip", "pointwise.hip"])
def test_no_lds_read_hoisted_above_a_barrier(src):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "barrier_hoist_check.py"), os.path.join(CSRC, src)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "total hoisted ds_reads: 0" in r.stdout, r.stdout + r.stderr
