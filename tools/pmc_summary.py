"""Average PMC counters per dispatch of the kernels matching a name filter, from every rocpd
DB under a rocprofv3 output directory (one DB per counter pass).

    python tools/pmc_summary.py gpurun_out/pmc_dir --kernel conv_igemm --min-us 500

HBM bytes: FETCH_SIZE / WRITE_SIZE are reported in KiB by rocprofv3; the MI355X guide's
gfx950 correction applies on top (roofline "traffic").
"""
import argparse
import collections
import glob
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for db in sorted(glob.glob(a.dir + "/**/*.db", recursive=True)):
        c = sqlite3.connect(db)
        q = """select name, dispatch_id, duration, counter_name, sum(counter_value) from pmc_events
               group by name, dispatch_id, counter_name"""
        for name, did, dur, cn, v in c.execute(q):
            if a.kernel not in name or dur / 1e3 < a.min_us:
                continue
            short = name.replace("_ZN12_GLOBAL__N_1", "")[:90]
            acc[short][cn].append(v)
            durs[short].append(dur / 1e3)
    for k, cs in acc.items():
        d = durs[k]
        print(f"## {k}  dispatches(all passes)={len(d)} avg_us={sum(d) / len(d):.1f}")
        for cn in sorted(cs):
            vs = cs[cn]
            print(f"   {cn:28s} {sum(vs) / len(vs):16.1f}")
        g = {cn: sum(v) / len(v) for cn, v in cs.items()}
        if "SQ_WAVE_CYCLES" in g and g["SQ_WAVE_CYCLES"]:
            w = g["SQ_WAVE_CYCLES"]
            for cn in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if cn in g:
                    print(f"   {cn + ' / WAVE_CYCLES':40s} {g[cn] / w:8.3f}")
        if "SQ_INSTS_LDS" in g and "SQ_LDS_BANK_CONFLICT" in g and "SQ_LDS_IDX_ACTIVE" in g and g["SQ_LDS_IDX_ACTIVE"]:
            print(f"   {'LDS bank-conflict / LDS active':40s} {g['SQ_LDS_BANK_CONFLICT'] / g['SQ_LDS_IDX_ACTIVE']:8.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in g and "GRBM_GUI_ACTIVE" in g and g["GRBM_GUI_ACTIVE"]:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back);
            # SQ_VALU_MFMA_BUSY_CYCLES = 16 x the 16x16x32 MFMAs issued (matrix-pipe cycles, all SIMDs)
            gui = g["GRBM_GUI_ACTIVE"] / 8
            print(f"   {'MFMA busy / (GUI_ACTIVE/8 * 1024 SIMD)':40s} {g['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui * 1024):8.3f}")
            print(f"   {'effective clock GHz (GUI_ACTIVE/8 / dur)':40s} {gui / (sum(d) / len(d) * 1e3):8.3f}")


if __name__ == "__main__":
    main()
