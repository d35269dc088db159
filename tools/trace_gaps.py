"""GPU idle time inside a traced bench run (rocprofv3 --kernel-trace rocpd DB): the union of all
kernel intervals over the span of the busiest window, and the largest idle gaps between them.
Answers whether host launch latency / synchronisation leaves the GPU idle (what a captured graph
would recover) or the step is kernel-bound.

    python tools/trace_gaps.py gpurun_out/x_tr/.../bench_results.db [--top 10]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=10)
    ap.add_argument("--split", type=float, default=5.0, help="ms of idle that separates segments")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = sorted(c.execute("""select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d
                               join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""))
    if not rows:
        print("no dispatches")
        return
    busy, gaps = 0, []
    cs, ce, prev_name = rows[0][0], rows[0][1], rows[0][2]
    for st, en, name in rows[1:]:
        if st > ce:
            busy += ce - cs
            gaps.append((st - ce, ce, prev_name[:60], name[:60]))
            cs, ce = st, en
        else:
            ce = max(ce, en)
        prev_name = name
    busy += ce - cs
    span = rows[-1][1] - rows[0][0]
    print(f"# {len(rows)} dispatches over {span / 1e6:.2f} ms: GPU busy {busy / 1e6:.2f} ms "
          f"({100 * busy / span:.1f} %), idle {(span - busy) / 1e6:.2f} ms in {len(gaps)} gaps")
    big = [g for g in gaps if g[0] > 1e6]                 # > 1 ms: between steps / host work
    small = [g for g in gaps if g[0] <= 1e6]
    print(f"# gaps <= 1 ms: {len(small)} totalling {sum(g[0] for g in small) / 1e6:.2f} ms; "
          f"> 1 ms: {len(big)} totalling {sum(g[0] for g in big) / 1e6:.2f} ms")
    for g in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g[0] / 1e3:9.1f} us after {g[2]}  ->  {g[3]}")
    # segments of back-to-back work (split at gaps > --split ms): the bench's timed steps are the
    # longest such segment (no host synchronisation inside the timed region)
    segs, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(x[1] for x in cur[-64:]) > a.split * 1e6:
            segs.append(cur)
            cur = [r]
        else:
            cur.append(r)
    segs.append(cur)
    print(f"# segments split at idle > {a.split} ms (longest first):")
    for sg in sorted(segs, key=lambda g: g[-1][1] - g[0][0], reverse=True)[:6]:
        span = max(x[1] for x in sg) - sg[0][0]
        b, cs, ce = 0, sg[0][0], sg[0][1]
        gap_list = []
        for st, en, _ in sg[1:]:
            if st > ce:
                b += ce - cs
                gap_list.append(st - ce)
                cs, ce = st, en
            else:
                ce = max(ce, en)
        b += ce - cs
        print(f"  {len(sg):6d} dispatches, span {span / 1e6:8.2f} ms, busy {b / 1e6:8.2f} ms "
              f"({100 * b / span:5.1f} %), {len(gap_list)} gaps, largest {max(gap_list, default=0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
