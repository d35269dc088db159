"""Write profiles/r02_pmc_traffic_<config>.json (the bench line's `traffic`) from two rocprofv3
PMC passes (FETCH_SIZE, WRITE_SIZE; kernel-trace only) over the dominant conv launch.

    python tools/traffic_json.py <fetch_dir> <write_dir> --kernel conv_halo --min-us 2000 \
        --layer vit_pose.adapter.7 --batch 256 --precision 0 --algorithmic <bytes> --out <json>

FETCH_SIZE / WRITE_SIZE are KiB (rocprofv3); on gfx950 FETCH_SIZE reports half the bytes of a
16-B-per-lane streaming read (MI355X_MICROARCH.md, HBM), so reads are FETCH_SIZE x 2 KiB.
"""
import argparse
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def avg_counter(d, counter, kernel, min_us):
    vals = []
    for db in sorted(glob.glob(d + "/**/*.db", recursive=True)):
        c = sqlite3.connect(db)
        q = """select name, dispatch_id, duration, sum(counter_value) from pmc_events where counter_name = ?
               group by name, dispatch_id"""
        for name, _, dur, v in c.execute(q, (counter,)):
            if kernel in name and dur / 1e3 >= min_us:
                vals.append((v, dur / 1e3, name))
    if not vals:
        raise SystemExit(f"no {counter} dispatches of {kernel} >= {min_us} us under {d}")
    return sum(v for v, _, _ in vals) / len(vals), sum(t for _, t, _ in vals) / len(vals), vals[0][2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--min-us", type=float, default=1000.0)
    ap.add_argument("--layer", required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--precision", type=int, required=True)
    ap.add_argument("--algorithmic", type=float, required=True, help="algorithmic HBM bytes per launch")
    ap.add_argument("--shape", default="")
    ap.add_argument("--command", default="tools/run_r02_final.sh")
    ap.add_argument("--sources", default="", help="comma list of the csrc files the kernel is built from")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import bench
    f, tf, name = avg_counter(a.fetch_dir, "FETCH_SIZE", a.kernel, a.min_us)
    w, tw, _ = avg_counter(a.write_dir, "WRITE_SIZE", a.kernel, a.min_us)
    rd, wr = f * 2 * 1024, w * 1024
    srcs = [x for x in a.sources.split(",") if x] or None
    out = {"kernel": name[:160], "layer": a.layer, "shape": a.shape, "batch": a.batch, "precision": a.precision,
           "fetch_size_kib": f, "write_size_kib": w,
           "correction": "FETCH_SIZE x2 (gfx950: half the bytes of 16-B-per-lane reads); WRITE_SIZE as reported",
           "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
           "algorithmic_bytes_per_launch": a.algorithmic, "avg_us_profiled": [round(tf, 1), round(tw, 1)],
           "sources": srcs, "sources_sha": bench.kernel_sources_hash(srcs),
           "command": f"{a.command} (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE --kernel-trace, separate passes)"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
