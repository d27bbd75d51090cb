"""Host model of the lane kernel (crc32c_kernels.hip, crc32c_lane_kernel):
one record per lane, 128-B line tasks, the schedule of issue() and fold().

For random runs of 64 records (lengths around the kernel's limits, any
alignment, records the kernel leaves to the generic path among them) the model
mirrors issue() step by step -- head bytes h, body words n4, tail bytes tb,
the body's first line vl and first word q0, the lane's last task kend, the
run's K and partial-line mask pm, the line a lane reads in task k -- and checks:

  * every body load is one whole 128-B line holding a byte of the lane's own
    record (a line with a record byte lies in a mapped page: no fault), and
    the head / end dwords lie inside the record's first / last 4-B word;
  * folding the loaded words with the kernel's masks (task 0: the register
    enters at word q0; tasks whose bit is clear in pm fold unmasked, kept
    only by lanes whose line is all body; tasks with the bit set fold masked
    word by word) and the edge bytes -- the head dword, a log header's crc and
    the tail bytes taken from the line registers where the line holds them,
    loaded otherwise -- gives the oracle's crc (oracle/crc32c_oracle.c, pinned
    to the reference's golden vectors).

CPU only: no device is touched."""
import numpy as np
import pytest

P = 0x82F63B78
MINLEN, MAXLEN = 8, 1280  # kLaneMinLen, kLaneMaxLen (crc32c_device.h)


def _shift_bytes(x, n):
    for _ in range(8 * n):
        x = (x >> 1) ^ (P if x & 1 else 0)
    return x


S = [[_shift_bytes(b << (8 * k), 4) for b in range(256)] for k in range(4)]  # slice4[k][b]


def step(a, w):  # step256 with the slice4 tables: shift_4(a) ^ w
    return w ^ S[0][a & 255] ^ S[1][(a >> 8) & 255] ^ S[2][(a >> 16) & 255] ^ S[3][a >> 24]


def byte_step(r, b):  # shift_1(r ^ b)
    y = r ^ b
    return S[3][y & 255] ^ (y >> 8)


def lane_run(buf, offs, lens, inits):
    """One run of 64 records through the kernel's schedule; returns
    ({lane: crc} for the lanes the kernel owns, list of load violations)."""
    u32 = lambda a: int.from_bytes(bytes(buf[a:a + 4]), "little")
    nl = len(offs)
    bad = []
    lanes = []
    for l in range(nl):
        p, ln = int(offs[l]), int(lens[l])
        owned = MINLEN <= ln <= MAXLEN
        h = (-p) & 3 if owned else 0
        n4 = (ln - h) >> 2 if owned else 0
        tb = (ln - h) & 3 if owned else 0
        vb = p + h
        q0 = (vb & 127) >> 2 if owned else 0
        qe = q0 + n4
        lanes.append(dict(p=p, ln=ln, owned=owned, h=h, n4=n4, tb=tb, vl=vb & ~127, q0=q0,
                          kend=(qe + 31) >> 5 if owned else 1, qe=qe))
    K = max(x["kend"] for x in lanes)
    pm = 0
    for x in lanes:
        if x["owned"] and x["qe"] & 31:
            pm |= 1 << (x["qe"] >> 5)
    acc = [0] * nl
    out = {}
    for k in range(K):
        for l, x in enumerate(lanes):
            if not x["owned"]:
                continue
            line = x["vl"] + 128 * min(k, x["kend"] - 1)
            if not (line % 128 == 0 and line < x["p"] + x["ln"] and line + 128 > x["p"]):
                bad.append(("line", l, k))
            w = [u32(line + 4 * i) for i in range(32)]
            a = acc[l]
            if k == 0:
                hd_addr = x["p"] & ~3
                if not (hd_addr <= x["p"] < hd_addr + 4):
                    bad.append(("head", l))
                # the head dword from the line (word q0 - 1), loaded only when the body starts the line
                hd = w[x["q0"] - 1] if x["q0"] else u32(hd_addr)
                if x["h"] and hd != u32(hd_addr):
                    bad.append(("head_pick", l))
                hb = hd >> (8 * ((4 - x["h"]) & 3))
                # a log header's crc (6 B before the span) from the line, loaded when it starts before it
                o = 4 * x["q0"] - x["h"] - 6
                if o >= 0 and x["p"] >= 6:
                    j, sh = o >> 2, o & 3
                    pair = w[j] | (w[min(j + 1, 31)] << 32)
                    if (pair >> (8 * sh)) & 0xFFFFFFFF != u32(x["p"] - 6):
                        bad.append(("crc_pick", l))
                r = inits[l] ^ 0xFFFFFFFF
                for i in range(3):
                    v = byte_step(r, (hb >> (8 * i)) & 255)
                    r = v if i < x["h"] else r
                for i in range(32):
                    rel = (i - x["q0"]) & 0xFFFFFFFF
                    y = r ^ w[i] if rel == 0 else step(a, w[i])
                    a = y if rel < x["n4"] else a
            elif not (pm >> k) & 1:
                y = a
                for i in range(32):
                    y = step(y, w[i])
                if 32 * k + 32 <= x["qe"]:
                    a = y
                elif 32 * k < x["qe"]:
                    bad.append(("clean", l, k))  # a partial line outside pm
            else:
                rel0 = (32 * k - x["q0"]) & 0xFFFFFFFF
                for i in range(32):
                    y = step(a, w[i])
                    a = y if ((rel0 + i) & 0xFFFFFFFF) < x["n4"] else a
            acc[l] = a
            if k + 1 == K:
                r = step(a, 0)
                ed_addr = x["p"] + x["ln"] - 4
                if ed_addr < x["p"]:
                    bad.append(("end", l))
                qe = x["qe"]
                fw = w[qe & 31] if qe & 31 else u32(ed_addr) >> (8 * ((4 - x["tb"]) & 3))
                fb = fw & ((1 << (8 * x["tb"])) - 1)
                if x["tb"] and fb != u32(ed_addr) >> (8 * (4 - x["tb"])):
                    bad.append(("tail_pick", l))
                for i in range(3):
                    v = byte_step(r, (fb >> (8 * i)) & 255)
                    r = v if i < x["tb"] else r
                out[l] = r ^ 0xFFFFFFFF
    return out, bad


@pytest.mark.parametrize("seed", range(6))
def test_lane_schedule_matches_oracle(oracle, seed):
    rng = np.random.default_rng(0x1A4E0000 + seed)
    size = 1 << 18
    buf = oracle.synth(size, 0x1A4E0000 + seed)
    kind = rng.integers(0, 4, size=64)
    lens = np.select([kind == 0, kind == 1, kind == 2],
                     [rng.integers(0, 24, size=64), rng.integers(990, 1032, size=64),
                      rng.integers(1281, 3000, size=64)],
                     rng.integers(MINLEN, MAXLEN + 1, size=64)).astype(np.uint64)
    if seed % 2:  # contiguous log-file layout: neighbours share lines
        offs = np.cumsum(np.concatenate([[int(rng.integers(0, 128))], (lens + 7)[:-1]])).astype(np.uint64)
    else:
        offs = rng.integers(0, size - 3000, size=64).astype(np.uint64)
    inits = rng.integers(0, 2**32, size=64, dtype=np.uint64).astype(np.uint32)
    out, bad = lane_run(buf, offs, lens, [int(v) for v in inits])
    assert not bad, bad[:5]
    want, _ = oracle.batch(buf, offs, lens, inits)
    owned = [l for l in range(64) if MINLEN <= int(lens[l]) <= MAXLEN]
    assert sorted(out) == owned
    for l in owned:
        assert out[l] == int(want[l]), (l, int(lens[l]), int(offs[l]))


def test_lane_every_line_position(oracle):
    """Every body start position within a line (q0 = 0..31, h = 0..3) and
    lengths that end at every position of the last line."""
    buf = oracle.synth(1 << 16, 0x1A4E00FF)
    offs = np.array([4096 + 128 * i + i % 128 for i in range(64)], dtype=np.uint64)
    for shift in (0, 1, 2, 3):
        o = offs + np.uint64(shift * 64 + 3 * shift)
        lens = np.array([MINLEN + (37 * i + 11 * shift) % (MAXLEN - MINLEN + 1) for i in range(64)], dtype=np.uint64)
        out, bad = lane_run(buf, o, lens, [0] * 64)
        assert not bad
        want, _ = oracle.batch(buf, o, lens)
        assert [out[l] for l in range(64)] == [int(v) for v in want]
