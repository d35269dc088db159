"""Per-kernel table of one PMC ratio over a whole program run (GPU box; reads the rocpd DBs of
a rocprofv3 --pmc run): for every kernel name, its dispatch count, total time, and the
duration-weighted mean of NUM / (GRBM_GUI_ACTIVE / 8) -- the fraction of the kernel's cycles a
per-CU unit counter such as TA_BUSY_avr (texture-address unit busy) was set. Sorted by the
time the unit was busy (total ms x fraction): the kernels where that unit is worth relieving.

    python tools/pmc_table.py gpurun_out/DIR --num TA_BUSY_avr [--top 40]
"""
import argparse
import collections
import glob
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--num", default="TA_BUSY_avr")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    per = collections.defaultdict(dict)                  # (name, dispatch) -> counter -> value
    dur = {}
    for db in sorted(glob.glob(a.dir + "/**/*.db", recursive=True)):
        c = sqlite3.connect(db)
        q = """select name, dispatch_id, duration, counter_name, sum(counter_value) from pmc_events
               group by name, dispatch_id, counter_name"""
        for name, did, d, cn, v in c.execute(q):
            per[(name, did)][cn] = v
            dur[(name, did)] = d / 1e6
    rows = collections.defaultdict(lambda: [0, 0.0, 0.0])   # name -> [n, ms, ms x frac]
    for key, cs in per.items():
        if a.num not in cs or not cs.get("GRBM_GUI_ACTIVE"):
            continue
        f = cs[a.num] / (cs["GRBM_GUI_ACTIVE"] / 8)
        r = rows[key[0]]
        r[0] += 1
        r[1] += dur[key]
        r[2] += dur[key] * f
    tot = sum(r[1] for r in rows.values())
    print(f"{a.num} / (GRBM_GUI_ACTIVE / 8), duration-weighted; {tot:.2f} ms of kernels in total")
    print("   busy-ms  total-ms   frac    n  kernel")
    for name, (n, ms, bf) in sorted(rows.items(), key=lambda kv: -kv[1][2])[:a.top]:
        short = name.replace("_ZN12_GLOBAL__N_1", "").replace("(anonymous namespace)::", "")[:110]
        print(f"  {bf:8.2f} {ms:9.2f} {bf / ms:6.3f} {n:4d}  {short}")


if __name__ == "__main__":
    main()
