"""Host model of the quad kernel's addressing (crc32c_kernels.hip, issue()):
every body word and edge byte a lane loads must be a byte of a record the
kernel owns (its body, its head/tail, the stored crc it verifies) or of the
zero block, for any batch geometry.  A GPU fault is the failure mode this
guards against; the model mirrors issue() step by step (window, row geometry,
body addresses max(bw + 4 i, bw - 256 m) + 256 m in 32-bit unsigned
arithmetic, the safe word of rows without body words, edge lanes).
CPU only: no device is touched."""
import numpy as np
import pytest

MAXLEN, QW, BACK = 1280, 320, 1280  # kQuadMaxLen, kQuadWords, kQuadBack (crc32c_device.h)
M32 = 0xFFFFFFFF
BASE = 0x7F00_0000_0000
ZERO = 0x10_0000_0000_0000  # stands for DeviceTables::zero


def quad_window(base, off, ln, valid):
    sh = [bool((valid >> q) & 1) and ln[q] <= MAXLEN for q in range(4)]
    if not any(sh):
        return 0, 0
    a = sh.index(True)
    aa = base + off[a] - BACK
    sb = aa - min(aa, 1 << 30)
    mask = 0
    for q in range(4):
        d = base + off[q] - sb
        if sh[q] and BACK <= d < (1 << 31) - 2048:
            mask |= 1 << q
    return sb, mask


def bad_loads(offs, lens, verify, hdr, base=BASE):
    n, bad = len(offs), 0
    for tb in range(0, n, 4):
        off = [int(offs[min(tb + q, n - 1)]) for q in range(4)]
        ln = [int(lens[min(tb + q, n - 1)]) for q in range(4)]
        valid = sum(1 << q for q in range(4) if tb + q < n)
        sb, mask = quad_window(base, off, ln, valid)
        rows = []
        for q in range(4):
            ok = bool((mask >> q) & 1)
            vpo = base + off[q] - sb if ok else 8
            h = min((-(sb + vpo)) & 3, ln[q])
            W, t = (ln[q] - h) >> 2, (ln[q] - h) & 3
            if not ok:
                W = h = t = 0
            rows.append((ok, vpo, h, W, t, ln[q]))
        withw = [r[3] > 0 for r in rows]
        sbase = sb if any(withw) else ZERO - BACK
        safe = rows[withw.index(True)][1] + rows[withw.index(True)][2] if any(withw) else BACK
        bodies = [(sb + r[1] + r[2], sb + r[1] + r[2] + 4 * r[3]) for r in rows if r[0] and r[3]]
        for q, (ok, vpo, h, W, t, L) in enumerate(rows):
            p = base + off[q]
            bo = vpo + h
            bw, P = (bo if W else safe), QW - W
            for m in range(5):
                for k in range(4):
                    for j in range(16):
                        ad = (bw + 4 * (16 * (k ^ (q & 1)) + j - P)) & M32
                        lo = (bw - 256 * m) & M32
                        addr = sbase + max(ad, lo) + 256 * m
                        good = sbase == ZERO - BACK and addr == ZERO
                        good = good or any(lo <= addr and addr + 4 <= hi for lo, hi in bodies)
                        bad += not good
            edges = [(p, p + L)] if ok else []
            if ok and verify:
                edges.append((p - 6, p) if hdr else (p + L, p + L + 4))
            for j in range(16):
                qd, o = j >> 2, j & 3
                ev, eo = False, 0
                if qd == 0:
                    ev, eo = o < h, vpo + o
                elif qd == 1:
                    ev, eo = o < t, bo + 4 * W + o
                elif qd == 2:
                    ev, eo = verify and ok, (vpo - 6 + o) if hdr else bo + 4 * W + t + o
                if ev:
                    bad += not any(lo <= sb + eo < hi for lo, hi in edges)
    return bad


@pytest.mark.parametrize("seed", range(6))
def test_quad_loads_stay_in_owned_records(seed):
    rng = np.random.default_rng(0x0ADD0000 + seed)
    n = int(rng.choice([1, 2, 3, 5, 63, 300]))
    lens = np.where(rng.random(n) < 0.7, rng.integers(0, 1300, size=n), rng.integers(0, 70_000, size=n))
    off = rng.integers(6, 64 << 20, size=n)
    if seed % 2:
        off[::3] += 3 << 30  # records of one task more than 2 GiB apart
    verify = bool(seed & 2)
    hdr = verify and bool(seed & 4) or seed == 5
    assert bad_loads(off, lens, verify, hdr) == 0


def test_window_leaves_far_and_long_records():
    """A task with a record 5 GiB away and a 100 000-byte one: both go to the
    generic path.  The window base lies 1 GiB below the anchor record, so a
    row the kernel does not own must not read at base + 8 (an earlier build
    did, and faulted): the model above checks that rows without body words
    read another row's body word instead."""
    off = np.array([1400, 5 << 30, 1600, 1800])
    lens = np.array([10, 10, 100_000, 20])
    sb, mask = quad_window(BASE, list(off), list(lens), 15)
    assert mask == 0b1001
    assert sb + 8 < BASE  # the read that faulted
