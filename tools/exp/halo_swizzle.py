"""Exhaustive search (container) for the 16-B slot swizzle of a haloed LDS tile (conv.h
swz_halo): find f(column) in 0..7 such that every 16-pixel fragment window the 3x3 taps read
(starting at column kw or 16 + kw of a halo row, kw = 0..2) puts the 16 lanes of each
ds_read_b128 lane group -- rows fr in {0-3, 12-15} at logical slot L, rows {4-11} at L ^ 2 --
on distinct (pixel parity, physical slot) pairs (MI355X_MICROARCH.md, LDS). Rows of 18 or 34
pixels start at even pixel indices, so the parity is the column's."""
A = {0, 1, 2, 3, 12, 13, 14, 15}


def ok_window(f, kw, ncols):
    seen = set()
    for fr in range(16):
        col = kw + fr
        if col >= ncols or f[col] is None:
            continue
        key = (col & 1, f[col] ^ (0 if fr in A else 2))
        if key in seen:
            return False
        seen.add(key)
    return True


def solve(ncols, kws):
    f = [None] * ncols

    def bt(i):
        if i == ncols:
            return True
        for v in range(8):
            f[i] = v
            if all(ok_window(f, kw, ncols) for kw in kws) and bt(i + 1):
                return True
        f[i] = None
        return False

    return f if bt(0) else None


if __name__ == "__main__":
    print("18 columns (8x16 / 16x16 tiles):", solve(18, [0, 1, 2]))
    print("34 columns (8x32 tile):", solve(34, [0, 1, 2, 16, 17, 18]))
    T = [0, 1, 4, 0, 1, 5, 4, 5]
    packed = sum(t << (3 * k) for k, t in enumerate(T))
    print("period-16 table", T, "packed", hex(packed))
