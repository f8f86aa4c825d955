"""Host check of the recomputing walk's window logic (ta_walk_ck.hip): the
walk of checkpoint plans crosses each 16-row stripe in windows that start at
the stripe's checkpoint column at least kCkLead columns left of the walk
(checkpoints at columns 16 (b + 1) - l for stripe lane l, or column 0), and
steps one row at a time -- stop on a cell with H = 0, else the run of I moves
(trailing ones of the row's I-only bits, stopped at the window's edge), then
the D or M move out of the row.  Here the same window arithmetic runs on the
exact DP matrix of the reference recurrence (team_alignment.cpp:171-217) and
must give the reference walk's path for every pair, including I runs longer
than a window and D runs across stripes."""
import numpy as np
import pytest

LEAD = 17


def dp(q, t, ma, mi, gap):
    n, m = len(q), len(t)
    H = np.zeros((n + 1, m + 1), np.int64)
    D = np.zeros((n + 1, m + 1), bool)
    I = np.zeros((n + 1, m + 1), bool)
    best, gi, gj = None, 0, 0
    for i in range(1, n + 1):
        for j in range(1, m + 1):
            dg = H[i - 1, j - 1] + (ma if q[i - 1] == t[j - 1] else mi)
            lf, up = H[i, j - 1] + gap, H[i - 1, j] + gap
            I[i, j], D[i, j] = lf > dg, up > max(dg, lf)
            H[i, j] = max(dg, lf, up, 0)
            if best is None or H[i, j] > best:
                best, gi, gj = H[i, j], i, j
    return H, D, I, gi, gj


def reference_walk(H, D, I, i, j):
    out = []
    while H[i, j] > 0:
        if D[i, j]:
            out.append("D")
            i -= 1
        elif I[i, j]:
            out.append("I")
            j -= 1
        else:
            out.append("M")
            i, j = i - 1, j - 1
    return "".join(reversed(out))


def window_walk(H, D, I, i, j, q, t, sc):
    """The kernel's walk: window columns and row steps; H only as the 0 test.
    Each window is first recomputed from its checkpoint column and the stripe
    above's bottom row alone, as the kernel does, and must equal the matrix."""
    out = []
    while True:
        g, r = (i - 1) >> 4, (i - 1) & 15
        lane = g & 63
        e = j - LEAD + lane
        c0 = max((e >> 4) * 16 - lane, 0) if e >= 16 else 0
        W = j - c0
        assert 1 <= W <= LEAD + 15 and c0 >= 0, (W, j, c0)
        ma, mi, gap = sc
        hw = {}
        for a in range(16 * g + 1, min(16 * g + 16, H.shape[0] - 1) + 1):
            for b in range(c0 + 1, j + 1):
                get = lambda u, v: H[u, v] if (u == 16 * g or v == c0) else hw[(u, v)]  # noqa: E731
                s = ma if q[a - 1] == t[b - 1] else mi
                hw[(a, b)] = max(get(a - 1, b - 1) + s, get(a, b - 1) + gap, get(a - 1, b) + gap, 0)
                assert hw[(a, b)] == H[a, b], (a, b)
        # row words: column x at bit W - x; I-only, D, zero
        rows = {}
        for rr in range(r + 1):
            a = 16 * g + rr + 1
            io = dd = zz = 0
            for x in range(1, W + 1):
                b, bit = c0 + x, 1 << (W - x)
                io |= bit if (I[a, b] and not D[a, b]) else 0
                dd |= bit if D[a, b] else 0
                zz |= bit if H[a, b] == 0 else 0
            rows[rr] = (io, dd, zz)
        rr, x, stop = r, W, False
        while rr >= 0 and x >= 1:
            io, dd, zz = rows[rr]
            pos = W - x
            if (zz >> pos) & 1:
                stop = True
                break
            v, run = io >> pos, 0
            while v & 1 and run < x:
                v >>= 1
                run += 1
            out += ["I"] * run
            x -= run
            if x == 0:
                break
            if (dd >> (pos + run)) & 1:
                out.append("D")
            else:
                out.append("M")
                x -= 1
            rr -= 1
        i, j = 16 * g + rr + 1, c0 + x
        if stop or i < 1 or j < 1:
            return "".join(reversed(out))


@pytest.mark.parametrize("sc", [(1, -1, -1), (2, -3, -1), (3, 4, 0), (4, -1, -2), (1, 0, -1)])
def test_window_walk_matches_reference(sc):
    rng = np.random.default_rng(0xC4 + sc[0] * 31 + sc[2])
    al = b"ACGT"
    # (the last two: stripes of lanes >= 16, whose first checkpoints precede column 1)
    for k, (n, m) in enumerate([(70, 90), (120, 60), (40, 130), (100, 100), (90, 75), (33, 140), (400, 45), (700, 30)]):
        q = bytes(al[v] for v in rng.integers(4, size=n))
        t = bytes(al[v] for v in rng.integers(4, size=m))
        if k % 3 == 1:  # a long insertion in the target: an I run longer than a window
            cut = n // 2
            t = (q[:cut] + b"N" * 45 + q[cut:])[:m] if m > cut + 45 else t
        if k % 3 == 2:  # a deletion: a D run across stripes
            cut = min(n, m) // 3
            q = (t[:cut] + b"N" * 35 + t[cut:])[:n]
        if k >= 6:  # the target is a piece of the query deep down: the path reaches column 1 there
            t = q[n - m - 20:n - 20]
        H, D, I, gi, gj = dp(q, t, *sc)
        if H[gi, gj] <= 0:
            continue
        assert window_walk(H, D, I, gi, gj, q, t, sc) == reference_walk(H, D, I, gi, gj), (sc, k)


def ck_row_index(pss, t, lane, nb):  # ta_layout.h
    return (pss * nb * 2 * 64 + (t >> 4) * 64 + lane) * 16 + (t & 15)


def ck_col_index(pss, b, lane, nb, r):
    return ((pss * 2 + 1) * nb * 64 + b * 64 + lane) * 16 + r


@pytest.mark.parametrize("n,m", [(1000, 1000), (1030, 990), (2100, 700), (40, 1200), (1500, 64), (300, 280),
                                 (1, 1), (17, 33), (1100, 1100)])
def test_window_loads_in_bounds(n, m):
    """Every HBM load of the walk kernel's window (traceback_ck_kernel, its
    index arithmetic restated for every cell (i, j) a walk can stand on and
    every lane of a group) lies inside the pair's checkpoint region, target and
    query, and the top-row loads of columns > 0 address ck_row_index of the
    stripe above exactly (block offsets of +1024 / +2048 from two bases)."""
    nb = (m + 63 + 15) // 16
    region = ((n + 1023) // 1024) * nb * 2048  # int16 entries (ptr_dwords_blk * 2)
    j = np.arange(1, m + 1, dtype=np.int64)
    for i in range(1, n + 1):
        g = (i - 1) >> 4
        l = g & 63
        e = j - LEAD + l
        c0 = np.where(e >= 16, np.maximum((e >> 4) * 16 - l, 0), 0)
        W = j - c0
        assert (W >= 1).all() and (W <= LEAD + 15).all()
        for lg in range(8):
            li = np.where(c0 > 0, ck_col_index(g >> 6, (e >> 4) - 1, l, nb, 2 * lg), 0)
            assert (li >= 0).all() and (li + 1 < region).all()
            if g > 0:
                gu = g - 1
                lu, pu = gu & 63, gu >> 6
                t0 = c0 + lg + lu - 1
                t1 = t0 + 8
                base = pu * nb * 2048 + lu * 16
                i0 = base + (t0 >> 4) * 1024 + (t0 & 15)
                i1 = base + (t1 >> 4) * 1024 + (t1 & 15)
                for q, idx in enumerate((np.maximum(i0, 0), i1, i0 + 1024, i1 + 1024, i0 + 2048)):
                    assert (idx >= 0).all() and (idx < region).all(), (n, m, i, lg, q)
                    col = c0 + lg + 8 * q
                    ok = col > 0
                    assert (idx[ok] == ck_row_index(pu, col[ok] + lu - 1, lu, nb)).all(), (n, m, i, lg, q)
            for q in range(4):
                x = 1 + lg + 8 * q
                tix = (c0 + x - 1)[x <= W]
                assert (tix >= 0).all() and (tix < m).all()
            assert 0 <= min(16 * g + 2 * lg + 1, n - 1) < n


def kernel_events_walk(H, D, I, i, j, q, t, sc):
    """The kernel's walk at the bit level (traceback_ck_kernel): per window the
    row words NI = ~I | D and D of W bits (column x at bit W - x), the row steps
    with the 33-bit run bound, records, the walk's cost from the records (H
    itself is never read but at the goal: the first record whose cell has cost 0
    ends the walk), and the events of the records with the I run carried across
    windows -- expanded into ops (walk order)."""
    ma, mi, gap = sc
    ev, kI, cost = [], 0, int(H[i, j])
    while True:
        g, r = (i - 1) >> 4, (i - 1) & 15
        lane = g & 63
        e = j - LEAD + lane
        c0 = max((e >> 4) * 16 - lane, 0) if e >= 16 else 0
        W = j - c0
        rows = {}
        for rr in range(r + 1):
            a = 16 * g + rr + 1
            iw = dw = 0
            for x in range(1, W + 1):
                b, bit = c0 + x, 1 << (W - x)
                iw |= bit if I[a, b] else 0
                dw |= bit if D[a, b] else 0
            rows[rr] = ((~iw | dw) & 0xFFFFFFFF, dw)
        pos, rr, wl, recs = 0, r, 1, []
        while wl:
            # (past a cell with H = 0 the walk goes on over whatever codes are there; the
            # records it lists after that are cut below)
            ni, dw = rows[rr] if rr in rows else (0, 0)
            v = (ni >> pos) | (1 << 32)
            run = min((v & -v).bit_length() - 1, W - pos)
            p1 = pos + run
            edge = 1 if p1 >= W else 0
            dmove = (dw >> (p1 & 31)) & 1
            mv = wl & (edge ^ 1)
            recs.append(run | (dmove << 8) | (edge << 9) | (p1 << 10))
            pos += run + (mv & (dmove ^ 1))
            rr -= mv
            wl = mv & (1 if rr >= 0 else 0) & (1 if pos < W else 0)
        # the cost before each record; the first record k >= 1 (k = len: after the last)
        # with cost 0 ends the walk
        hk, zstop = [cost], False
        for k, rc in enumerate(recs):
            ed, dm, x = rc & 0x200, rc & 0x100, W - ((rc >> 10) & 63)
            s = (ma if q[16 * g + r - k] == t[c0 + x - 1] else mi) if not ed and not dm else 0
            hk.append(hk[-1] - gap * ((rc & 63) + (1 if not ed and dm else 0)) - s)
        for k in range(1, len(recs) + 1):
            if hk[k] == 0:
                recs, zstop = recs[:k], True
                break
        cost = hk[len(recs)]
        # M moves with no I run between them: one event at the run's last record
        mm = zm = 0
        for k, rc in enumerate(recs):
            runI = (rc & 63) + (kI if k == 0 else 0)
            mm |= (1 if (rc & 0x300) == 0 else 0) << k
            zm |= (1 if runI == 0 else 0) << k
        cont = mm & zm & (mm << 1)
        for k, rc in enumerate(recs):
            runI = (rc & 63) + (kI if k == 0 else 0)
            if rc & 0x200:
                continue
            if runI:
                ev.append((runI << 2) | 1)
            if rc & 0x100:
                ev.append((1 << 16) | 3)
            elif not (cont >> (k + 1)) & 1:
                below = ~cont & ((2 << k) - 1)
                ev.append((k + 1 - (below.bit_length() - 1)) << 2)
        if recs:
            last = recs[-1]
            kI = ((last & 63) + (kI if len(recs) == 1 else 0)) if last & 0x200 else 0
        i, j = 16 * g + rr + 1, c0 + W - pos
        if zstop or i < 1 or j < 1:
            break
    ops = []
    for v in ev:
        kd, bc, mop = v >> 16, (v >> 2) & 0x3FFF, v & 3
        ops += ["D"] * kd
        if mop != 3:
            ops += ["MID"[mop]] * bc
    return "".join(reversed(ops))


@pytest.mark.parametrize("sc", [(1, -1, -1), (2, -3, -1), (3, 4, 0)])
def test_kernel_events_walk_matches_reference(sc):
    """The bit-level walk and its events give the reference path, including I
    runs that cross several 32-column windows (the run bound of a full window)."""
    rng = np.random.default_rng(0xE7 + sc[0])
    al = b"ACGT"
    for k, (n, m, ins) in enumerate([(120, 200, 70), (90, 160, 45), (70, 90, 0), (200, 150, 33), (60, 140, 64)]):
        q = bytes(al[v] for v in rng.integers(4, size=n))
        t = bytes(al[v] for v in rng.integers(4, size=m))
        if ins:
            cut = n // 2
            t = (q[:cut] + b"N" * ins + q[cut:] + t)[:m]
        H, D, I, gi, gj = dp(q, t, *sc)
        if H[gi, gj] <= 0:
            continue
        assert kernel_events_walk(H, D, I, gi, gj, q, t, sc) == reference_walk(H, D, I, gi, gj), (sc, k)
