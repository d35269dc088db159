"""Summarise a rocprofv3 --kernel-trace results DB (rocpd sqlite) per kernel name.

    python tools/prof_summary.py gpurun_out/prof1/r01_results.db [--passes 3] > profiles/x.txt
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--passes", type=int, default=1, help="forward passes in the trace (for per-pass ms)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    q = """select s.kernel_name, count(*), sum(d.end-d.start), avg(d.end-d.start), min(d.end-d.start),
                  max(d.end-d.start), s.arch_vgpr_count, s.accum_vgpr_count, s.group_segment_size
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.kernel_name order by 3 desc"""
    rows = list(c.execute(q))
    tot = sum(r[2] for r in rows)
    print(f"# rocprofv3 --kernel-trace summary of {a.db}")
    print(f"# total kernel time {tot / 1e6:.2f} ms over {a.passes} pass(es) = {tot / 1e6 / a.passes:.2f} ms/pass")
    print(f"{'total_ms':>10} {'ms/pass':>9} {'%':>6} {'calls':>6} {'avg_us':>10} {'min_us':>9} {'max_us':>10}"
          f" {'vgpr':>5} {'agpr':>5} {'lds':>7}  kernel")
    for r in rows:
        name = r[0].replace("_ZN12_GLOBAL__N_1", "").replace(".kd", "")
        print(f"{r[2] / 1e6:10.2f} {r[2] / 1e6 / a.passes:9.2f} {100 * r[2] / tot:6.2f} {r[1]:6d} {r[3] / 1e3:10.1f}"
              f" {r[4] / 1e3:9.1f} {r[5] / 1e3:10.1f} {r[6]:5d} {r[7]:5d} {r[8]:7d}  {name[:120]}")


if __name__ == "__main__":
    main()
