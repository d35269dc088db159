"""Compare tools/layer_profile.py outputs layer by layer (min over repeats of each variant).

    python tools/lp_compare.py A:file1,file2 B:file3,file4 [--filter backbone]
"""
import re
import sys


def load(files):
    best = {}
    for f in files:
        for line in open(f):
            m = re.match(r"\s*([\d.]+)\s+[\d.]+\s+[\d.]+\s+\d\s+.*?\s(\S+) x\d+$", line)
            if m:
                ms, name = float(m.group(1)), m.group(2)
                best[name] = min(best.get(name, 1e9), ms)
    return best


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    if flt in args:
        args.remove(flt)
    vs = [(a.split(":")[0], load(a.split(":")[1].split(","))) for a in args]
    names = sorted(vs[0][1], key=lambda n: -vs[0][1][n])
    print(f"{'layer':45s} " + " ".join(f"{v:>9s}" for v, _ in vs))
    tot = [0.0] * len(vs)
    for n in names:
        if flt and flt not in n:
            continue
        row = [d.get(n, float("nan")) for _, d in vs]
        tot = [t + r for t, r in zip(tot, row)]
        if max(row) - min(row) > 0.02:
            print(f"{n:45s} " + " ".join(f"{r:9.3f}" for r in row))
    print(f"{'total (' + (flt or 'all') + ')':45s} " + " ".join(f"{t:9.3f}" for t in tot))


if __name__ == "__main__":
    main()
