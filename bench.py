"""Benchmark: whole-node frames/s of the per-frame multi-task hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config full|yolo_face|yolo_raw|vitpose] [--batch B]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

Configs (BASELINE.json ``configs``; the bench line is config 4 by default):
  full       config 4 (config 5 at N = 8): 256 synthetic 640x640 frames per GPU, resident in
             HBM; ResNet-50 trunk once -> face-YOLO (det [B,5,525], strides 8/16/32) + AdaFace
             (emb, norm) + ViTPose-B (heatmaps) -> batched NMS (padded, on device) + heatmap
             soft-argmax; for N > 1 the per-rank frame records (padded detections, embeddings,
             keypoints) are all-gathered over RCCL (the only exchange).
  yolo_face  config 2: 64 frames per GPU, trunk -> face-YOLO -> NMS.
  yolo_raw   config 2's kernel micro-bench variant: YOLO v11n nc=1 straight on
             64 raw 640x640 frames per GPU (A = 8400) -> NMS.
  vitpose    config 3: 256 pixel_values crops [3,256,192] per GPU -> ViTPose-B -> soft-argmax.
Frames shard across ranks (each rank owns a contiguous slice of the global batch), weights are
replicated, no collective on the data path; value = all ranks' frames / max-over-ranks time
("weak" scaling).

Multi-GPU launch: with ``--gpus N > 1`` and no WORLD_SIZE in the environment, this process
starts N child processes (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, 127.0.0.1)
BEFORE it touches the GPU, waits for them and exits with their status; rank 0 prints the line.
Under torchrun the ranks come from the environment.

Rank 0 prints ONE JSON line. Extra objects:
  roofline     — the dominant kernel of the config, timed with HIP events on its stream
                 (isolated pass right after the timed region when the heads run concurrently;
                 its in-region, co-resident time is reported beside it); achieved = its
                 algorithmic FLOPs per launch / mean launch time; peak = dense bf16 MFMA 2.5 PF/s.
                 ``traffic`` (HBM bytes per launch, PMC FETCH_SIZE x2 + WRITE_SIZE) comes from the
                 newest committed profiles/rNN_pmc_traffic_<config>.json only while the sources of that
                 kernel (the files listed there) hash to the value recorded there (else null,
                 "stale").
  cpu_baseline — the oracle (fp32 PyTorch-CPU restatement of the reference, pinned against the
                 reference itself) on this host's usable cores: warm-up 1, median of 5, at
                 bs=1 and bs=8 (value = the bs=8 rate). A reported baseline, not the target.
  parity       — the GPU outputs vs that CPU reference on frames spread over the batch
                 (0, B/3, 2B/3, B-1): heatmaps / embeddings max|d|, keypoint OKS delta (max
                 over the sampled frames), NMS exactness on the sampled frames.
For N > 1 the full config all-gathers each frame's record (padded detections + count,
embedding + norm, keypoints + scores: 9.5 KB per frame) in one collective per step.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "person-recognition-for-pose-estimation_amd")]

METRIC = "frames/sec whole-node, 640×640 bs=256, 1/2/4/8 MI355X; OKS Δ vs CPU ref"
MFMA_BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
STRIDE = [8.0, 16.0, 32.0]
CONFIGS = {
    # name: (default per-GPU batch, dominant pack(s) for the roofline line, BASELINE config, workload)
    "full": (256, ["vit_pose.adapter.7"], 4,
             "full multi-task model (trunk + face-YOLO + AdaFace + ViTPose + NMS + soft-argmax), 640x640"),
    "yolo_face": (64, ["yolo_face.adapter.10"], 2, "YOLO-face detection head (trunk + face-YOLO + NMS), 640x640"),
    "yolo_raw": (64, ["yolo_face.yolo.net.p1.0"], 2,
                 "YOLO v11n nc=1 on raw 640x640 frames (config-2 micro-bench variant, A=8400) + NMS"),
    "vitpose": (256, [f"vit_pose.vit_pose.backbone.encoder.layer.{i}:fc1" for i in range(12)], 3,
                "ViTPose-B keypoint head on 256x192 crops (pixel_values -> heatmaps -> soft-argmax)"),
}
DTYPE = ("f32 storage/accumulate; split-operand MFMA: trunk 2x fp16 planes (3 terms), YOLO net 3x bf16 "
         "(6 terms), YOLO / ViT adapters and ViT 2x bf16 (3 terms), AdaFace adapter 3x3s + IR-50 1x fp16 "
         "plane with per-frame power-of-2 scaling (1 term)")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="full", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="frames per GPU (0 = the config's)")
    ap.add_argument("--precision", default="auto")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--sequential-heads", action="store_true",
                    help="enqueue the three heads on one stream (default: one HIP stream per head)")
    ap.add_argument("--dominant", default="", help="pack name(s) timed for the roofline (comma list)")
    return ap.parse_args()


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_children(n: int, cmd: list[str] | None = None) -> int:
    """One child process per GPU (no GPU call in this process): ``cmd`` (default: this script
    with the same arguments) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT set; returns the first non-zero exit status (then the other ranks are killed)."""
    port = _free_port()
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    try:
        for p in procs:
            p.wait()
            rc = rc or p.returncode
            if p.returncode:          # one rank failed: the others would block in a collective
                for q in procs:
                    if q.poll() is None:
                        q.kill()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


# ----------------------------------------------------------------------------- helpers
def usable_cores() -> int:
    """CPUs this process may run on: the affinity set, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def kernel_sources_hash(names=None) -> str:
    """Hash of the kernel sources (csrc/*.hip, *.h), or of just ``names`` (the files the
    measured kernel is built from, e.g. ["conv_halo.hip", "conv.h", "common.h"])."""
    h = hashlib.sha256()
    pkg = os.path.join(ROOT, "person-recognition-for-pose-estimation_amd", "csrc")
    files = sorted(glob.glob(os.path.join(pkg, "*.hip")) + glob.glob(os.path.join(pkg, "*.h")))
    if names:
        files = sorted(os.path.join(pkg, n) for n in names)
    for f in files:
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def spread(B: int) -> list[int]:
    return sorted({0, B // 3, (2 * B) // 3, B - 1})


def conv_flops(p, pixels):
    return 2.0 * pixels * p.co * p.ci * p.kh * p.kw


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_children(args.gpus))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:
        dist.init_process_group("nccl", device_id=dev)
        observed_ws = dist.get_world_size()
    else:
        observed_ws = 1

    from prpe import CombinedModel, arch, ops, synth
    from prpe.dist import gather_detections, gather_frame_records, gather_tensor
    from prpe.postproc import non_max_suppression_padded

    cfg = args.config
    B0, dominant, cfg_no, workload = CONFIGS[cfg]
    B = args.batch or B0
    dominant = args.dominant.split(",") if args.dominant else dominant
    prec = args.precision if args.precision == "auto" else int(args.precision)
    sd = synth.make_state_dict(arch.state_dict_spec())
    model = CombinedModel(sd, device=dev, precision=prec)
    eng = model.engine
    eng.prepare()
    if cfg == "vitpose":
        x = synth.uniform(100 + rank, f"pixel_values:{B}x256x192", (B, 3, 256, 192)).to(dev)
    else:
        x = synth.frames(B, seed=100 + rank).to(dev)

    def step():
        if cfg == "full":
            o = model.forward_all(x, face_stride=STRIDE, concurrent=not args.sequential_heads)
            dets, cnt = non_max_suppression_padded(o["det"])
            coords, scores = ops.softargmax(o["heatmaps"])
            o.update(dets=dets, cnt=cnt, coords=coords)
            if ws > 1:
                # one RCCL all-gather over xGMI of each frame's record: detections + count,
                # embedding + norm, keypoints + scores (prpe/dist.py)
                o["gathered"] = gather_frame_records([dets, cnt, o["emb"], o["norm"],
                                                      torch.cat([coords, scores[..., None]], -1)])
        elif cfg == "yolo_raw":
            det = eng.yolo_raw("yolo_face", x, STRIDE)
            dets, cnt = non_max_suppression_padded(det)
            o = {"det": det, "dets": dets, "cnt": cnt}
            if ws > 1:
                gather_detections(dets, cnt)
        elif cfg == "yolo_face":
            det = eng.yolo("yolo_face", eng.trunk(x), STRIDE)
            dets, cnt = non_max_suppression_padded(det)
            o = {"det": det, "dets": dets, "cnt": cnt}
            if ws > 1:
                gather_detections(dets, cnt)
        else:
            heat = model.vitpose_from_pixels(x).heatmaps
            coords, scores = ops.softargmax(heat)
            o = {"heatmaps": heat, "coords": coords}
            if ws > 1:
                gather_tensor(torch.cat([coords, scores[..., None]], -1))
        return o

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.watch = set(dominant)
    eng.events = {}
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        o = step()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    eng.watch = set()
    if ws > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    fps = B * ws * args.steps / elapsed

    # ---- roofline of the dominant kernel. With the heads on their own streams the dominant
    # launch shares the CUs with the other heads' kernels, so its event time inside the timed
    # region measures co-residence: it is reported as "in_timed_region_ms" and the roofline line
    # comes from an isolated pass (heads sequential, same kernels and shapes) right after.
    def ev_ms(evs):
        return [a.elapsed_time(b) for a, b, *_ in evs]

    timed = [m for d in dominant for m in ev_ms(eng.events.get(d, []))]
    isolated = cfg == "full" and not args.sequential_heads
    if isolated:
        eng.events = {}
        eng.watch = set(dominant)
        for _ in range(3):
            model.forward_all(x, face_stride=STRIDE, concurrent=False)
        torch.cuda.synchronize(dev)
        eng.watch = set()
    evs = [e for d in dominant for e in eng.events.get(d, [])]
    roof = None
    if evs:
        ms = ev_ms(evs)
        _, _, pixels, p, precn, x_numel = evs[0]
        avg_s = sum(ms) / len(ms) / 1e3
        fl = conv_flops(p, pixels)
        passes = {0: 3, 1: 1, 2: 6, 3: 3}[precn]
        name = dominant[0] if len(dominant) == 1 else dominant[0].replace(".layer.0:", ".layer.*:")
        kern = (f"prpe_conv2d[{name}] {p.kh}x{p.kw}/{p.stride} {p.ci}->{p.co} "
                f"(library's automatic kernel/tile choice, precision {precn})")
        # algorithmic bytes: the input read once, the output written once, the fp32 weights once
        nbytes = 4.0 * (x_numel + pixels * p.co + p.co * p.ci * p.kh * p.kw)
        # the bound: whichever of the two rates the launch runs closer to ITS peak -- HBM bytes / s
        # against 8 TB/s, or the MFMA work it executes (algorithmic FLOPs x the split's passes)
        # against the dense bf16 peak (a flop/byte ridge on fp32 bytes called ViT fc1
        # "hbm" at 1.1 TB/s)
        hbm_frac = nbytes / avg_s / 1e9 / HBM_PEAK_GBS
        mfma_exec_frac = fl * passes / avg_s / 1e12 / MFMA_BF16_PEAK_TFLOPS
        if hbm_frac > mfma_exec_frac:
            ach = nbytes / avg_s / 1e9
            roof = {"bound": "hbm", "kernel": kern, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_gb_per_launch": round(nbytes / 1e9, 4),
                    "flop_per_byte": round(fl / nbytes, 2)}
        else:
            ach = fl / avg_s / 1e12
            roof = {"bound": "mfma", "kernel": kern, "achieved": round(ach, 2), "peak": MFMA_BF16_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / MFMA_BF16_PEAK_TFLOPS, 4),
                    "executed_mfma_passes": passes, "executed_frac": round(ach * passes / MFMA_BF16_PEAK_TFLOPS, 4)}
        roof.update({"bound_rule": "larger of hbm_frac, mfma_executed_frac", "hbm_frac": round(hbm_frac, 4),
                     "mfma_executed_frac": round(mfma_exec_frac, 4)})
        roof.update({"avg_launch_ms": round(sum(ms) / len(ms), 4), "launches": len(ms),
                "measured": ("isolated pass after the timed region (heads sequential)" if isolated
                             else "inside the timed region"),
                "in_timed_region_ms": round(sum(timed) / len(timed), 4) if timed else None,
                "algorithmic_gflop_per_launch": round(fl / 1e9, 2), "traffic": None})
        recs = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc_traffic_{cfg}.json")))
        tp = recs[-1] if recs else ""                    # the newest round's record
        if tp:
            t = json.load(open(tp))
            fresh = (t.get("sources_sha") == kernel_sources_hash(t.get("sources")) and t.get("batch") == B
                     and t.get("layer") in dominant and t.get("precision") == precn)
            if fresh:
                roof["traffic"] = round(t["hbm_bytes_per_launch"] / 1e9, 3)
                roof["traffic_unit"] = ("GB per launch, L2-to-fabric bytes incl. Infinity-Cache hits "
                                        "(PMC FETCH_SIZE x2 + WRITE_SIZE)")
                roof["algorithmic_gb_per_launch"] = round(t["algorithmic_bytes_per_launch"] / 1e9, 3)
                roof["traffic_source"] = os.path.relpath(tp, ROOT)
            else:
                roof["traffic_source"] = f"stale ({os.path.relpath(tp, ROOT)} was collected on other kernel sources)"

    # ---- parity on frames spread over the batch + CPU baseline, rank 0, N = 1 only
    cpu = parity = None
    if rank == 0 and not args.no_cpu_baseline and ws == 1:
        parity, cpu = cpu_legs(cfg, sd, x, o, B, args.cpu_reps)
    # ---- N > 1 (full config): rank 0 checks the records the timed region's all-gather delivered
    # for sampled frames of EVERY rank's shard against the oracle on those frames (regenerated
    # from the rank's input seed); each rank contributes its sampled frames' raw det rows (one
    # more small all-gather, outside the timed region) so NMS exactness is checked on them
    if ws > 1 and cfg == "full" and not args.no_cpu_baseline:
        det_samples = gather_tensor(o["det"][sample_local(B)].contiguous())
        if rank == 0:
            from oracle import model_ref as R
            torch.set_num_threads(usable_cores())
            recs = [t.cpu() for t in o["gathered"]]
            parity = gathered_parity(recs, det_samples.cpu(), B, ws, sd, R,
                                     lambda r, idx: synth.frame_rows(B, idx, seed=100 + r))

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(fps, 2), "unit": "frames/sec" if cfg != "vitpose" else "crops/sec",
            "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": DTYPE,
            "data": "synthetic (splitmix64 frames U[0,1), seeded weights + calibrated BN; no network)",
            "config": {"workload": workload, "baseline_config": cfg_no, "global_batch": B * ws, "per_gpu_batch": B,
                       "parallelism": f"dp{ws} (frame sharding, RCCL all-gather of detections)",
                       "world_size_observed": observed_ws, "precision_policy": str(args.precision)},
            "roofline": roof, "cpu_baseline": cpu, "parity": parity,
            "oks_delta": parity.get("oks_delta") if parity else None,
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()


def sample_local(B: int) -> list[int]:
    """Frames of each rank's shard whose gathered records rank 0 checks at N > 1."""
    return sorted({0, B // 2, B - 1})


def gathered_parity(recs, det_samples, B, ws, sd, R, frames_of, stride=STRIDE):
    """Config 5 parity: the all-gathered frame records (dets [G,300,6], cnt [G], emb [G,512],
    norm [G,1], keypoints + scores [G,17,3], G = B*ws, rank order) on the sampled frames of
    every rank's shard vs the oracle ``R`` on the same frames (``frames_of(r, idx)`` regenerates
    rank r's inputs): keypoint OKS delta and embedding max|d| against the oracle forward, and
    NMS rows exact against the oracle NMS of the rank's own det rows (``det_samples``
    [ws*len(idx), 5, A], gathered in rank order)."""
    import torch
    dets, cnt, emb, _norm, kp = recs
    idx = sample_local(B)
    out = {"frames": [], "oks_delta": 0.0, "emb_max_abs": 0.0, "cls_max_abs": 0.0, "nms_exact": True,
           "checked": "all-gathered records of sampled frames of every rank vs the oracle"}
    with torch.no_grad():
        for r in range(ws):
            g = [r * B + i for i in idx]
            ds = det_samples[r * len(idx):(r + 1) * len(idx)]
            ref = R.forward_all(sd, frames_of(r, idx), stride=stride)
            rc, _ = R.keypoints_from_heatmaps(ref["heatmaps"])
            out["oks_delta"] = max(out["oks_delta"], R.oks_delta(kp[g][..., :2], rc))
            out["emb_max_abs"] = max(out["emb_max_abs"], float((emb[g] - ref["emb"]).abs().max()))
            out["cls_max_abs"] = max(out["cls_max_abs"], float((ds[:, 4] - ref["det"][:, 4]).abs().max()))
            for j, m in enumerate(R.non_max_suppression(ds)):
                out["nms_exact"] &= int(cnt[g[j]]) == len(m) and bool(torch.equal(dets[g[j], :len(m)], m))
            out["frames"] += g
    return out


def cpu_legs(cfg, sd, x, o, B, reps):
    """(parity, cpu_baseline): the oracle on this host (test infrastructure, after the timed
    region; the product path never imports it)."""
    import torch
    from oracle import model_ref as R
    threads = usable_cores()
    torch.set_num_threads(threads)
    idx = spread(B)
    xs = x[idx].cpu()
    parity = {"frames": idx}
    with torch.no_grad():
        if cfg == "full":
            ref = R.forward_all(sd, xs, stride=STRIDE)
            parity["heatmaps_max_abs"] = float((o["heatmaps"][idx].cpu() - ref["heatmaps"]).abs().max())
            parity["emb_max_abs"] = float((o["emb"][idx].cpu() - ref["emb"]).abs().max())
            parity["cls_max_abs"] = float((o["det"][idx, 4].cpu() - ref["det"][:, 4]).abs().max())
            rc, _ = R.keypoints_from_heatmaps(ref["heatmaps"])
            parity["oks_delta"] = R.oks_delta(o["coords"][idx].cpu(), rc)
        elif cfg == "yolo_face":
            det = R.yolo_branch(sd, "yolo_face", R.resnet50_trunk(sd, xs), STRIDE)
            parity["cls_max_abs"] = float((o["det"][idx, 4].cpu() - det[:, 4]).abs().max())
        elif cfg == "yolo_raw":
            det = R.yolo_net(sd, "yolo_face", xs, STRIDE)
            parity["cls_max_abs"] = float((o["det"][idx, 4].cpu() - det[:, 4]).abs().max())
        else:
            heat = R.vitpose_backbone(sd, xs)
            parity["heatmaps_max_abs"] = float((o["heatmaps"][idx].cpu() - heat).abs().max())
            rc, _ = R.keypoints_from_heatmaps(heat)
            parity["oks_delta"] = R.oks_delta(o["coords"][idx].cpu(), rc)
        if "dets" in o:
            # NMS bit-exact on the same det tensor (sampled frames)
            mine = R.non_max_suppression(o["det"][idx].cpu())
            cnt = o["cnt"][idx].cpu()
            dets = o["dets"][idx].cpu()
            parity["nms_exact"] = all(int(cnt[i]) == len(m) and torch.equal(dets[i, :len(m)], m)
                                      for i, m in enumerate(mine))

    def run(xb):
        with torch.no_grad():
            if cfg == "full":
                r = R.forward_all(sd, xb, stride=STRIDE)
                R.non_max_suppression(r["det"])
                R.keypoints_from_heatmaps(r["heatmaps"])
            elif cfg == "yolo_face":
                R.non_max_suppression(R.yolo_branch(sd, "yolo_face", R.resnet50_trunk(sd, xb), STRIDE))
            elif cfg == "yolo_raw":
                R.non_max_suppression(R.yolo_net(sd, "yolo_face", xb, STRIDE))
            else:
                R.keypoints_from_heatmaps(R.vitpose_backbone(sd, xb))

    rates = {}
    for bs in (1, 8):
        xb = x[:bs].cpu()
        run(xb)                                   # warm-up
        ts = []
        for _ in range(reps):
            t1 = time.perf_counter()
            run(xb)
            ts.append(time.perf_counter() - t1)
        rates[bs] = bs / statistics.median(ts)
    unit = "crops/sec" if cfg == "vitpose" else "frames/sec"
    cpu = {"value": round(rates[8], 4), "unit": unit, "cores": threads, "kind": "port",
           "sample": f"oracle (fp32 torch CPU restatement of the reference), warm-up 1 + median of {reps} "
                     f"at bs=8 (value) and bs=1 ({rates[1]:.4f} {unit}), same workload as the GPU step",
           "bs1": round(rates[1], 4)}
    return parity, cpu


if __name__ == "__main__":
    main()
