"""Phase timeline of the fused bottleneck (GPU box; measurement only): loads
tools/abl/libprpe_trace.so (tools/bneck_trace_build.py) in place of libprpe.so, runs the
layer1 (mid 64) and layer2 (mid 128) identity blocks at bs = 256, and reads back wave 0's
phase timestamps of every workgroup (100-MHz device clock).

Prints per phase the median / mean duration of one tile, and per CU the time-weighted mix of
phases its resident workgroups are in (1 = x loads + W1 MFMAs, e1 = t1 epilogue, 2 = 3x3 MFMAs
on LDS, e2 = t2 epilogue, 3 = W3 MFMAs + residual + y stores).

    python tools/bneck_trace.py [--batch 256]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from prpe import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "tools", "abl", "libprpe_trace.so")
from prpe import ops  # noqa: E402

SLOTS = 64
NAMES = ["1", "e1", "2", "e2", "3"]


def steps(tr, nk1):
    """per phase-1 K-step: wait (previous step's MFMA issue end -> past this step's barrier),
    split (past the barrier -> A(kt) landed and split), rest (-> next step's barrier)"""
    t0 = tr[:, 0].astype(np.int64) & 0xFFFFFFFF
    ts = (tr[:, 8:8 + nk1].astype(np.int64) - t0[:, None]) % (1 << 32)
    tss = (tr[:, 8 + nk1:8 + 2 * nk1].astype(np.int64) - t0[:, None]) % (1 << 32)
    tm = (tr[:, 8 + 2 * nk1:8 + 3 * nk1].astype(np.int64) - t0[:, None]) % (1 << 32)
    print("   phase-1 K-steps (median us):  kt: barrier-at  wait+barrier  split(A landed)  mfma issue")
    prev = np.zeros(len(tr), np.int64)
    for k in range(nk1):
        print(f"     {k:2d}: {np.median(ts[:, k]) / 100:7.2f} {np.median(ts[:, k] - prev) / 100:8.2f} "
              f"{np.median(tss[:, k] - ts[:, k]) / 100:8.2f} {np.median(tm[:, k] - tss[:, k]) / 100:8.2f}")
        prev = tm[:, k]


def analyse(tr, label, nk1):
    t = tr[:, :6].astype(np.int64)
    t -= t[:, 0].min()
    d = np.diff(t, axis=1)                      # [nwg, 5] phase durations in 10-ns ticks
    span = t[:, 5].max()
    print(f"== {label}: {len(t)} workgroups, kernel span {span / 100:.1f} us")
    print("   phase      median us   mean us   share of tile")
    tot = d.sum(1).mean()
    for k, nm in enumerate(NAMES):
        print(f"   {nm:>5}   {np.median(d[:, k]) / 100:10.2f} {d[:, k].mean() / 100:9.2f}   {d[:, k].mean() / tot:6.3f}")
    print(f"   tile    {np.median(d.sum(1)) / 100:10.2f} {tot / 100:9.2f}")
    steps(tr, nk1)
    hw, xcc = tr[:, 6].astype(np.int64), tr[:, 7].astype(np.int64)
    cu = (xcc & 0xF) * 256 + ((hw >> 8) & 0xFF)
    ucu = np.unique(cu)
    print(f"   CUs seen {len(ucu)}; workgroups per CU {len(t) / len(ucu):.1f}")
    # time-weighted phase mix per CU, sampled every 0.1 us
    step = 10
    grid = np.arange(0, span, step)
    mix = {}
    conc = np.zeros(4)
    for c in ucu[:64]:                          # 64 CUs is plenty for the statistics
        idx = np.where(cu == c)[0]
        ph = np.full((len(idx), len(grid)), -1, np.int8)
        for r, i in enumerate(idx):
            for k in range(5):
                a, b = np.searchsorted(grid, [t[i, k], t[i, k + 1]])
                ph[r, a:b] = k
        active = (ph >= 0).sum(0)
        for n in range(4):
            conc[n] += (active == n).sum()
        # for the instants with two resident workgroups: the unordered pair of phases
        two = np.where(active == 2)[0]
        if len(two):
            pp = np.sort(np.where(ph[:, two] >= 0, ph[:, two], 99), axis=0)[:2]
            keys, cnt = np.unique(pp[0] * 10 + pp[1], return_counts=True)
            for k_, n_ in zip(keys, cnt):
                mix[k_] = mix.get(k_, 0) + n_
    conc /= conc.sum()
    print("   resident workgroups per CU (time share): " + "  ".join(f"{n}: {conc[n]:.3f}" for n in range(4)))
    if mix:
        tot2 = sum(mix.values())
        print("   with two resident, phase pairs (time share):")
        for k_, n_ in sorted(mix.items(), key=lambda kv: -kv[1])[:10]:
            print(f"     ({NAMES[k_ // 10]:>2}, {NAMES[k_ % 10]:>2})  {n_ / tot2:.3f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    L = _lib.lib()
    L.prpe_bneck_trace_read.restype = C.c_int
    L.prpe_bneck_trace_read.argtypes = [C.c_void_p, C.c_ulonglong]
    from test_gpu_bneck import _packs, _packs128  # noqa: E402
    for mid in (64, 128):
        _, _, packs = _packs128(600) if mid == 128 else _packs(400)
        hw, c = (80, 512) if mid == 128 else (160, 256)
        g = torch.Generator("cuda").manual_seed(1)
        x = torch.relu(torch.randn(a.batch, hw, hw, c, generator=g, device="cuda"))
        xa = x.abs().flatten(1).amax(1).contiguous()
        y = torch.empty_like(x)
        ya = torch.zeros(a.batch, device="cuda")
        for _ in range(3):
            ops.bottleneck(x, packs, y, xa, ya)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.bottleneck(x, packs, y, xa, ya)
        e1.record()
        torch.cuda.synchronize()
        nwg = a.batch * ((hw + 15) // 16) * ((hw + 7) // 8)
        buf = np.zeros((nwg, SLOTS), np.uint64)
        rc = L.prpe_bneck_trace_read(buf.ctypes.data, buf.nbytes)
        assert rc == 0, rc
        analyse(buf, f"mid {mid} identity, bs {a.batch}, launch {e0.elapsed_time(e1):.3f} ms", 4 * mid // 32)
        del x, y


if __name__ == "__main__":
    main()
