"""Benchmark: whole-node frames/s of the per-frame multi-task hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256] [--config full]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = one pass of the hot path over one batch of synthetic 640x640 frames resident in
HBM (BASELINE.json config 4 per GPU; config 5 at N=8): ResNet-50 trunk once -> face-YOLO
(det [B,5,525], strides 8/16/32) + AdaFace (emb, norm) + ViTPose-B (heatmaps) -> batched
NMS (padded, on device) + heatmap soft-argmax; for N > 1 the per-rank padded detections are
all-gathered over RCCL (the only exchange). Frames are sharded: 256 per rank,
no collective on the data path; value = all ranks' frames / max-over-ranks time ("weak").

Rank 0 prints ONE JSON line. Extra objects:
  roofline     — the dominant kernel (largest conv launch), timed with HIP events on its
                 stream; with concurrent heads (default) in an isolated pass right after the
                 timed region (its in-region, co-resident time is reported beside it);
                 achieved = its algorithmic FLOPs per launch / mean launch time; peak = dense
                 bf16 MFMA 2.5 PF/s (the kernel runs split-bf16 MFMA; executed passes are
                 reported beside it).
  cpu_baseline — the oracle (fp32 PyTorch-CPU restatement of the reference, validated
                 bit-exact against the reference itself) on this host's cores, bounded sample.
  oks_delta    — keypoint OKS delta vs that CPU reference on the sampled frame.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "frames/sec whole-node, 640×640 bs=256, 1/2/4/8 MI355X; OKS Δ vs CPU ref"
MFMA_BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU")
    ap.add_argument("--precision", default="auto")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sequential-heads", action="store_true",
                    help="enqueue the three heads on one stream (default: one HIP stream per head)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--dominant", default="vit_pose.adapter.7",
                    help="conv pack timed with HIP events for the roofline line")
    return ap.parse_args()


def setup_dist(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if ws > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return ws, rank, local


def conv_flops(p, pixels):
    return 2.0 * pixels * p.co * p.ci * p.kh * p.kw


def main():
    args = parse()
    ws, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    from prpe import CombinedModel, arch, synth
    from prpe.postproc import non_max_suppression_padded
    from prpe.dist import gather_detections
    from prpe import ops

    prec = args.precision if args.precision == "auto" else int(args.precision)
    sd = synth.make_state_dict(arch.state_dict_spec())
    model = CombinedModel(sd, device=dev, precision=prec)
    eng = model.engine
    eng.prepare()
    B = args.batch
    x = synth.frames(B, seed=100 + rank).to(dev)
    stride = [8.0, 16.0, 32.0]

    def step():
        o = model.forward_all(x, face_stride=stride, concurrent=not args.sequential_heads)
        dets, cnt = non_max_suppression_padded(o["det"])
        coords, scores = ops.softargmax(o["heatmaps"])
        if ws > 1:
            gather_detections(dets, cnt)          # RCCL all-gather over xGMI (prpe/dist.py)
        return o, coords

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.watch = {args.dominant}
    eng.events = {}
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        o, coords = step()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    eng.watch = set()
    if ws > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    frames = B * ws * args.steps
    fps = frames / elapsed

    # ---- roofline of the dominant kernel. With the heads on their own streams the dominant
    # launch shares the CUs with the other heads' kernels, so its event time inside the timed
    # region measures co-residence, not the kernel: it is reported as "in_timed_region_ms" and
    # the roofline line itself comes from an isolated pass (heads sequential, same kernels and
    # shapes) run right after the timed region.
    ev_timed = eng.events.get(args.dominant, [])
    timed_ms = [a.elapsed_time(b) for a, b, *_ in ev_timed]
    isolated = not args.sequential_heads
    if isolated:
        eng.events = {}
        eng.watch = {args.dominant}
        for _ in range(3):
            model.forward_all(x, face_stride=stride, concurrent=False)
        torch.cuda.synchronize(dev)
        eng.watch = set()
    ev = eng.events.get(args.dominant, [])
    roof = None
    if ev:
        ms = [a.elapsed_time(b) for a, b, *_ in ev]
        _, _, pixels, p, precn = ev[0]
        avg_s = sum(ms) / len(ms) / 1e3
        fl = conv_flops(p, pixels)
        passes = {0: 3, 1: 1, 2: 6}[precn]
        ach = fl / avg_s / 1e12
        roof = {"bound": "mfma", "kernel": f"prpe_conv2d[{args.dominant}] {p.kh}x{p.kw} {p.ci}->{p.co} "
                                           f"(conv_wave_kernel, auto tile)",
                "achieved": round(ach, 2), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / MFMA_BF16_PEAK_TFLOPS, 4),
                "executed_mfma_passes": passes,
                "executed_frac": round(ach * passes / MFMA_BF16_PEAK_TFLOPS, 4),
                "avg_launch_ms": round(sum(ms) / len(ms), 4), "launches": len(ms),
                "measured": ("isolated pass after the timed region (heads sequential)" if isolated
                             else "inside the timed region"),
                "in_timed_region_ms": round(sum(timed_ms) / len(timed_ms), 4) if timed_ms else None,
                "algorithmic_gflop_per_launch": round(fl / 1e9, 2), "traffic": None}
        # HBM bytes per launch from the PMC passes committed under profiles/ (same kernel, layer
        # and batch; rocprofv3 cannot run inside this process): tools/run_traffic.sh
        tp = os.path.join(ROOT, "profiles", "r01_pmc_traffic_dominant.json")
        if os.path.exists(tp) and B == 256 and args.dominant == "vit_pose.adapter.7":
            t = json.load(open(tp))
            roof["traffic"] = round(t["hbm_bytes_per_launch"] / 1e9, 3)
            roof["traffic_unit"] = "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)"
            roof["algorithmic_gb_per_launch"] = round(t["algorithmic_bytes_per_launch"] / 1e9, 3)
            roof["traffic_source"] = "profiles/r01_pmc_traffic_dominant.json"

    # ---- CPU baseline (oracle restatement of the reference) + OKS delta, rank 0, N=1 only
    cpu = None
    oks = None
    if rank == 0 and not args.no_cpu_baseline and ws == 1:
        from oracle import model_ref as R
        nthreads = min(16, os.cpu_count() or 1)
        torch.set_num_threads(nthreads)
        x0 = x[:1].cpu()
        n = 0
        t1 = time.perf_counter()
        with torch.no_grad():
            while True:
                ref = R.forward_all(sd, x0, stride=stride)
                R.non_max_suppression(ref["det"])
                rc, _ = R.keypoints_from_heatmaps(ref["heatmaps"])
                n += 1
                if time.perf_counter() - t1 >= args.cpu_seconds:
                    break
        ct = time.perf_counter() - t1
        cpu = {"value": round(n / ct, 4), "unit": "frames/sec", "cores": nthreads, "kind": "port",
               "sample": f"{n} x 1 frame 640x640, full forward_all + NMS + soft-argmax, fp32 torch CPU"}
        oks = R.oks_delta(coords[:1].cpu(), rc)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(fps, 2), "unit": "frames/sec", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32 (split-bf16 MFMA)",
            "data": "synthetic (splitmix64 frames U[0,1), seeded weights + calibrated BN; no network)",
            "config": {"workload": "full multi-task model (trunk + face-YOLO + AdaFace + ViTPose + NMS + "
                                   "soft-argmax), 640x640", "global_batch": B * ws, "per_gpu_batch": B,
                       "parallelism": f"dp{ws} (frame sharding, RCCL all-gather of detections)",
                       "precision_policy": str(args.precision)},
            "roofline": roof, "cpu_baseline": cpu, "oks_delta": oks,
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
