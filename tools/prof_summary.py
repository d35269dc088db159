"""Summarise a rocprofv3 --kernel-trace results DB (rocpd sqlite) per kernel name.

    python tools/prof_summary.py gpurun_out/prof1/r01_results.db [--passes 3] > profiles/x.txt
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--passes", type=int, default=1, help="forward passes in the trace (for per-pass ms)")
    ap.add_argument("--dominant", default="%conv_wave%", help="SQL LIKE pattern of the dominant kernel")
    ap.add_argument("--grid", type=int, default=0, help="its grid size in work-items (0 = the largest)")
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
    if a.dominant:
        try:
            dominant(c, a.dominant, grid=a.grid)
        except sqlite3.Error as e:          # schema differences between rocprofv3 versions
            print(f"# dominant dispatch listing unavailable: {e}")


def dominant(c, name_like, limit=12, grid=0):
    """Per-dispatch durations of the largest grid among the kernels matching name_like (the bench's
    dominant conv launch): in the bench's default mode its first launches run inside the timed
    region beside the other heads (co-resident), the last ones in the isolated roofline pass."""
    q = """select d.grid_size_x * d.grid_size_y * d.grid_size_z as g, d.end - d.start, d.start, s.kernel_name
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           where s.kernel_name like ? order by g desc, d.start"""
    rows = list(c.execute(q, (name_like,)))
    if not rows:
        return
    g0 = grid if grid else rows[0][0]
    ds = [r for r in rows if r[0] == g0][:limit]
    print(f"# dominant dispatch (grid {g0} work-items, {ds[0][3][:80]}): durations in launch order, us")
    print("#   " + " ".join(f"{r[1] / 1e3:.1f}" for r in ds))


if __name__ == "__main__":
    main()
