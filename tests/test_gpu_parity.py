"""Parity of the MI355X engine against the oracle and the reference's golden
outputs.  Bit-exact (integer path).  All calls go through the C ABI
(prismdb_amd.crc32c -> libprismdb_crc32c.so)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001


@pytest.fixture(scope="module")
def dev(native):
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    from prismdb_amd import crc32c

    crc32c.device_init(0)
    return torch.device("cuda", 0)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _last_split(native):
    """{long spans, segments, overflow flag, lane-listed spans} of this thread's
    last planner-path descriptor batch (test hook prismdb_crc32c_last_split)."""
    import ctypes

    arr = (ctypes.c_uint64 * 4)()
    assert native.prismdb_crc32c_last_split(arr) == 0
    return list(arr)


def _to_dev(arr, dev):
    import torch

    return torch.from_numpy(np.array(arr, copy=True)).to(dev)


def test_golden_sweep_device(dev, golden, route):
    """Every reference golden vector (lengths 0..130 at offsets 0..7, block-sized
    spans, adversarial random spans, non-zero init) through batch()."""
    from prismdb_amd import crc32c

    buf = _to_dev(np.frombuffer(golden["input"], dtype=np.uint8), dev)
    rows = np.array(golden["vectors"]["rows"], dtype=np.uint64)
    off = _to_dev(rows[:, 0].astype(np.int64), dev)
    lens = _to_dev(rows[:, 1].astype(np.uint32).view(np.int32), dev)
    init = _to_dev(rows[:, 2].astype(np.uint32).view(np.int32), dev)
    out, _ = crc32c.batch(buf, off, lens, init)
    assert (_u32(out) == rows[:, 3].astype(np.uint32)).all()
    outm, _ = crc32c.batch(buf, off, lens, init, mask=True)
    assert (_u32(outm) == rows[:, 4].astype(np.uint32)).all()


def test_kats_device(dev, golden, route):
    from prismdb_amd import crc32c

    vecs = golden["kat"]["vectors"]
    blob = b"".join(bytes.fromhex(v["hex"]) for v in vecs) + b"\0" * 8
    offs, pos = [], 0
    for v in vecs:
        offs.append(pos)
        pos += len(v["hex"]) // 2
    buf = _to_dev(np.frombuffer(blob, dtype=np.uint8), dev)
    off = _to_dev(np.array(offs, dtype=np.int64), dev)
    lens = _to_dev(np.array([len(v["hex"]) // 2 for v in vecs], dtype=np.int32), dev)
    out, _ = crc32c.batch(buf, off, lens)
    assert crc32c.as_u32(out) == [v["value"] for v in vecs]


def test_long_stream_vectors_device(dev, golden, route):
    """Index-block sized spans (486 977 B), 1 MiB span: the split + combine path."""
    import torch
    from prismdb_amd import crc32c

    for s in golden["stream"]:
        a0 = s["byte_offset"] - s["byte_offset"] % 8
        buf = torch.empty(s["len"] + 16, dtype=torch.uint8, device=dev)
        crc32c.fill_synthetic(buf, s["seed"], a0)
        off = torch.tensor([s["byte_offset"] - a0], dtype=torch.int64, device=dev)
        lens = torch.tensor([s["len"]], dtype=torch.int32, device=dev)
        out, _ = crc32c.batch(buf, off, lens)
        assert crc32c.as_u32(out) == [s["crc"]], s


@pytest.fixture(params=["fast", "generic"])
def kernel_path(request, native):
    """Run fixed-stride cases through the fixed-geometry kernel and, forced,
    through the generic span kernel."""
    import ctypes

    native.prismdb_crc32c_force_generic.argtypes = [ctypes.c_int]
    native.prismdb_crc32c_force_generic(1 if request.param == "generic" else 0)
    yield request.param
    native.prismdb_crc32c_force_generic(0)


def test_fixed_4k_blocks_vs_oracle(dev, oracle, kernel_path):
    """Config-2 shape (4 KiB blocks, stride 4096) at 64 Ki blocks, all checked."""
    import torch
    from prismdb_amd import crc32c

    nblk, L = 1 << 16, 4096
    buf = torch.empty(nblk * L, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, SEED)
    host = oracle.synth(nblk * L, SEED)
    assert (buf[: 1 << 20].cpu().numpy() == host[: 1 << 20]).all()  # device generator == host generator
    want = oracle.batch_fixed(host, L, L, nblk)
    out, _ = crc32c.batch_fixed(buf, L, L, nblk)
    assert (_u32(out) == want).all()
    wantm = oracle.batch_fixed(host, L, L, nblk, init=0x12345678, mask=True)
    outm, _ = crc32c.batch_fixed(buf, L, L, nblk, init=0x12345678, mask=True)
    assert (_u32(outm) == wantm).all()


@pytest.mark.parametrize("stride,length", [(4096, 4095), (3992, 3988), (3993, 3988), (64, 61), (8192, 7),
                                           (1, 1), (4096, 0), (300000, 262147), (4096, 4), (4096, 256),
                                           (4100, 260), (2048, 2044), (8, 8), (4, 4), (12, 8), (5000, 4092)])
def test_fixed_odd_geometries(dev, oracle, stride, length, kernel_path):
    import torch
    from prismdb_amd import crc32c

    nblk = max(1, min(4096, (8 << 20) // max(stride, 1)))
    total = (nblk - 1) * stride + length + 8
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0005)
    host = buf.cpu().numpy()
    want = oracle.batch_fixed(host, stride, length, nblk, init=7)
    out, _ = crc32c.batch_fixed(buf, stride, length, nblk, init=7)
    assert (_u32(out) == want).all()


def _check_spans(dev, oracle, host, off, lens, init=None, mask=False):
    import torch
    from prismdb_amd import crc32c

    buf = _to_dev(host, dev)
    d_off = _to_dev(np.asarray(off, dtype=np.int64), dev)
    d_len = _to_dev(np.asarray(lens, dtype=np.uint32).view(np.int32), dev)
    d_init = _to_dev(np.asarray(init, dtype=np.uint32).view(np.int32), dev) if init is not None else None
    out, _ = crc32c.batch(buf, d_off, d_len, d_init, mask=mask)
    want, _ = oracle.batch(host, off, lens, init, mask=mask)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)


def test_mixed_sizes_config3(dev, oracle, route):
    """Config-3 shape: lengths uniform over {1,4,16,64} KiB packed back to back."""
    rng = np.random.default_rng(0x5EED0003)
    lens = rng.choice([1024, 4096, 16384, 65536], size=3000).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    host = oracle.synth(int(lens.sum()) + 16, 0x5EED0003)
    _check_spans(dev, oracle, host, off, lens)


def test_sst_shaped_config(dev, oracle, route):
    """SST-shaped: 3988-B spans at stride 3992 plus one 486 977-B index span."""
    n = 2000
    off = [i * 3992 for i in range(n)] + [n * 3992]
    lens = [3988] * n + [486977]
    host = oracle.synth(n * 3992 + 486977 + 16, 0x5EED0006)
    _check_spans(dev, oracle, host, off, lens, mask=True)


def test_adversarial_random_spans(dev, oracle, route):
    """Random lengths 0..70 000 at random byte offsets, random init (overlapping allowed)."""
    rng = np.random.default_rng(0x5EED0007)
    size = 8 << 20
    host = oracle.synth(size, 0x5EED0007)
    n = 5000
    lens = rng.integers(0, 70000, size=n).astype(np.uint64)
    off = (rng.integers(0, size - 70001, size=n)).astype(np.uint64)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    _check_spans(dev, oracle, host, off, lens, init)


def test_tiny_and_empty_spans(dev, oracle, route):
    host = oracle.synth(1 << 16, 0x5EED0008)
    off, lens = [], []
    for n in range(0, 40):
        for o in range(0, 9):
            off.append(1000 + 97 * n + o)
            lens.append(n)
    _check_spans(dev, oracle, host, off, lens, init=[(i * 2654435761) & 0xFFFFFFFF for i in range(len(off))])


def test_huge_span_split_path(dev, oracle, route):
    """A 40 MiB span at an odd offset (1281 segments) and neighbours."""
    size = (40 << 20) + 4096
    host = oracle.synth(size, 0x5EED0009)
    _check_spans(dev, oracle, host, [3, 17, (40 << 20) + 5], [40 << 20, 131073, 4000])


@pytest.mark.parametrize("n", [1 << 18, (1 << 18) + 1, 300001])
def test_pair_run_schedule(dev, oracle, native, n, bulk_route):
    """Batches the pair-run span kernel takes on the planner path (>= 2^18
    spans, every span one task), and the same batches as windows of the
    one-launch kernel: random lengths 0..4096 at random offsets, one in 997 a long span
    (split path) instead, per-span init, Mask, VERIFY with every seventh
    trailer damaged; odd counts leave an odd last run."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED0040 + n)
    lens = rng.integers(0, 4097, size=n).astype(np.int64)
    lens[::997] = rng.integers(131073, 400000, size=len(lens[::997]))
    slots = lens + 4
    off = np.concatenate([[11], 11 + np.cumsum(slots + rng.integers(0, 9, size=n))[:-1]]).astype(np.uint64)
    size = int(off[-1] + lens[-1] + 4 + 8)
    host = oracle.synth(size, 0x5EED0041)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    raw, _ = oracle.batch(host, off, lens.astype(np.uint32), init)
    masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    damaged = np.zeros(n, dtype=bool)
    damaged[3::7] = True
    stored = masked ^ damaged.astype(np.uint32)
    tr = (off + lens.astype(np.uint64)).astype(np.int64)[:, None] + np.arange(4)[None, :]
    host[tr] = stored.astype("<u4").view(np.uint8).reshape(-1, 4)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev)
    out, mm = crc32c.batch(buf, d_off, d_len, d_init, mask=True, verify=True)
    sched = (ctypes.c_uint64 * 3)()
    native.prismdb_crc32c_last_schedule.argtypes = [ctypes.c_void_p]
    rc = native.prismdb_crc32c_last_schedule(sched)
    if bulk_route == "planner":  # every record one task: the pair-run kernel's schedule, and it was launched
        assert rc == 0 and sched[0] == n and sched[1] == 0 and sched[2] == 1, (rc, list(sched))
    else:
        assert rc == -2  # windows of the one-launch kernel
    np.testing.assert_array_equal(_u32(out), masked)
    np.testing.assert_array_equal(mm.cpu().numpy(), damaged.astype(np.uint8))
    out2, _ = crc32c.batch(buf, d_off, d_len)  # no init / mask / verify
    np.testing.assert_array_equal(_u32(out2), oracle.batch(host, off, lens.astype(np.uint32))[0])
    # seal (MASK | WRITE_TRAILER) over zeroed trailers: every trailer is the
    # masked crc again and no other byte moves
    sealed = host.copy()
    sealed[tr] = 0
    sbuf = torch.from_numpy(sealed).to(dev)
    out3, _ = crc32c.batch(sbuf, d_off, d_len, d_init, mask=True, trailer=True)
    np.testing.assert_array_equal(_u32(out3), masked)
    want = sealed.copy()
    want[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
    np.testing.assert_array_equal(sbuf.cpu().numpy(), want)


def test_planner_seal_trailer_pass_without_out(dev, oracle, native, planner_bulk):
    """A sealing planner-path batch (300 001 spans: the pair-run kernel, long
    spans through the segment pass) with out = NULL: the trailer pass reads
    the results from the workspace's scratch.  Every trailer is the masked
    crc, no other byte moves; LOG_HEADER seals (header crc 6 bytes before
    each span) the same way on the span-only route."""
    import torch

    n = 300001
    rng = np.random.default_rng(0x5EED0042)
    lens = rng.integers(0, 4097, size=n).astype(np.int64)
    lens[5::1999] = rng.integers(131073, 300000, size=len(lens[5::1999]))
    off = np.concatenate([[19], 19 + np.cumsum(lens + 4 + 6 + rng.integers(0, 5, size=n))[:-1]]).astype(np.uint64)
    size = int(off[-1] + lens[-1] + 4 + 8)
    host = oracle.synth(size, 0x5EED0043)
    masked, _ = oracle.batch(host, off, lens.astype(np.uint32), mask=True)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    native.leveldb_crc32c_last_error.restype = ctypes.c_char_p
    for hdr in (False, True):
        prev = native.prismdb_crc32c_lane_mode(-1) if hdr else None  # log records without the lane kernel
        try:
            at = (off.astype(np.int64) - 6) if hdr else (off + lens.astype(np.uint64)).astype(np.int64)
            tr = at[:, None] + np.arange(4)[None, :]
            img = host.copy()
            img[tr] = 0
            buf = torch.from_numpy(img).to(dev)
            rc = native.leveldb_crc32c_batch(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
                                             ctypes.c_void_p(d_len.data_ptr()), None, ctypes.c_size_t(n), None, None,
                                             ctypes.c_uint32(0x3 | (0x4 if hdr else 0)),
                                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, native.leveldb_crc32c_last_error()
            want = img.copy()
            want[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
            got = buf.cpu().numpy()
            assert (got == want).all(), (hdr, np.nonzero(got != want)[0][:8])
        finally:
            if hdr:
                native.prismdb_crc32c_lane_mode(0)


@pytest.mark.parametrize("n", [1000, 300000])
def test_fixed_stride_seal(dev, oracle, native, n):
    """leveldb_crc32c_batch_fixed with MASK | WRITE_TRAILER (the generic path
    and its trailer pass: 4092-B contents||type blocks at stride 4096, and
    3987-B blocks at an odd stride), trailers zeroed first: afterwards every
    byte equals the oracle-sealed image and out holds the masked crcs."""
    import torch

    for stride, length in ((4096, 4092), (3993, 3987)):
        img = oracle.synth(n * stride + 8, 0x5EED0044 + stride)
        off = np.arange(n, dtype=np.uint64) * stride
        tr = (off + length).astype(np.int64)[:, None] + np.arange(4)[None, :]
        img[tr] = 0
        masked, _ = oracle.batch(img, off, np.full(n, length, dtype=np.uint32), mask=True)
        buf = torch.from_numpy(img).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        rc = native.leveldb_crc32c_batch_fixed(ctypes.c_void_p(buf.data_ptr()), stride, length, n, 0,
                                               ctypes.c_void_p(out.data_ptr()), None, ctypes.c_uint32(0x3),
                                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
        np.testing.assert_array_equal(_u32(out), masked)
        want = img.copy()
        want[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
        assert (buf.cpu().numpy() == want).all(), (stride, length)


def test_max_length_span(dev, oracle, native, route):
    """The longest span a descriptor holds (len = 2^32 - 1) at an odd offset,
    with an initial value, Mask and VERIFY against its stored trailer, next to
    a short span with a damaged trailer: the split path's 131 072 segments and
    their combine, against the oracle on host-regenerated bytes.  (The
    planner's segment and task counts wrapped in 32 bits for spans within
    32 KiB of 2^32.)"""
    import torch
    from prismdb_amd import crc32c

    L = 0xFFFFFFFF
    off = np.array([5, 5 + L + 4], dtype=np.uint64)
    lens = np.array([L, 1000], dtype=np.uint32)
    size = int(off[1]) + 1000 + 4 + 3
    free, _ = torch.cuda.mem_get_info()
    if free < size + (2 << 30):
        pytest.skip("not enough device memory for a 4 GiB span")
    seed = 0x5EED0031
    host = oracle.synth(size, seed)
    init = np.array([0x9E3779B9, 0x01234567], dtype=np.uint32)
    raw, _ = oracle.batch(host, off, lens, init)  # one pass over the 4 GiB (no trailer inside a span)
    want = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    for i, bad in ((0, 0), (1, 1)):
        t = int(off[i]) + int(lens[i])
        host[t:t + 4] = np.frombuffer(np.uint32(int(want[i]) ^ bad).tobytes(), dtype=np.uint8)
    buf = torch.empty(size, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, seed)
    for i in range(2):
        t = int(off[i]) + int(lens[i])
        buf[t:t + 4] = torch.from_numpy(host[t:t + 4].copy()).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32).copy()).to(dev)
    d_init = torch.from_numpy(init.view(np.int32).copy()).to(dev)
    out, mm = crc32c.batch(buf, d_off, d_len, d_init, mask=True, verify=True)
    np.testing.assert_array_equal(_u32(out), want)
    assert mm.cpu().numpy().tolist() == [0, 1]
    if route == "lane_log":
        assert _last_split(native)[:3] == [1, 131072, 0]  # one long span, 2^17 segments, no overflow
    out2, _ = crc32c.batch(buf, d_off[:1], d_len[:1], d_init[:1])  # unmasked, no verify
    assert int(_u32(out2)[0]) == int(raw[0])
    del buf, out, mm, out2
    torch.cuda.empty_cache()


def test_segment_workspace_overflow_fallback(dev, oracle, native, planner_bulk):
    """More long spans than the segment workspace lists (kCapLong = 2^18):
    the planner flags the overflow and the span pass folds every long span
    itself as a chain of 4 KiB chunks (no segment pass, no combine).  2^18 +
    64 spans of 128 KiB + 1 B (just above kLongSpan), one per 131 080-B
    stride with their stored trailers (34 GB), VERIFY with a per-span init,
    three trailers damaged.  Every other span is 65 536 B longer (49 chunks
    against 33): the fallback chains then have different lengths, which the
    pair-run schedule (one task per record) must not take."""
    import torch
    from prismdb_amd import crc32c

    S, L, L2, n = 196624, 131073, 196609, (1 << 18) + 64
    free, _ = torch.cuda.mem_get_info()
    if free < n * S + (4 << 30):
        pytest.skip("not enough device memory for the overflow case")
    pat = oracle.synth(2 * S, 0x5EED0032)  # two stride blocks, repeated
    init = 0x2468ACE1
    want = [oracle.mask(int(c)) for c in oracle.batch(pat, [0, S], [L, L2], [init, init])[0]]
    pat[L:L + 4] = np.frombuffer(np.uint32(want[0]).tobytes(), dtype=np.uint8)
    pat[S + L2:S + L2 + 4] = np.frombuffer(np.uint32(want[1]).tobytes(), dtype=np.uint8)
    buf = torch.empty(n * S, dtype=torch.uint8, device=dev)
    buf.view(n // 2, 2 * S).copy_(torch.from_numpy(pat).to(dev).expand(n // 2, 2 * S))
    lens = np.where(np.arange(n) % 2 == 0, L, L2)
    damaged = [0, 777, n - 1]
    for k in damaged:
        buf[k * S + int(lens[k]) + 2] ^= 0x40
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * S
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_init = torch.full((n,), init - (1 << 32) if init >= 1 << 31 else init, dtype=torch.int32, device=dev)
    out, mm = crc32c.batch(buf, d_off, d_len, d_init, mask=True, verify=True)
    assert _last_split(native)[2] == 1  # the workspace overflowed: the fallback ran
    got = _u32(out)
    wantv = np.where(np.arange(n) % 2 == 0, want[0], want[1]).astype(np.uint32)
    assert (got == wantv).all(), np.flatnonzero(got != wantv)[:10]
    m = mm.cpu().numpy()
    assert np.flatnonzero(m).tolist() == damaged
    # Sealing the same batch: the overflow again, and the trailer pass then
    # writes the long spans' trailers too (no combine to leave them to) --
    # the three damaged trailers are rewritten, the rest rewritten unchanged.
    out, _ = crc32c.batch(buf, d_off, d_len, d_init, mask=True, trailer=True)
    assert _last_split(native)[2] == 1
    assert (_u32(out) == wantv).all()
    _, mm = crc32c.batch(buf, d_off, d_len, d_init, mask=True, verify=True)
    assert int(mm.sum().item()) == 0
    del buf, d_off, d_len, d_init, out, mm
    torch.cuda.empty_cache()


@pytest.mark.parametrize("uniform", [False, True])
def test_long_spans_close_slices(dev, oracle, uniform, bulk_route):
    """300 000 short spans with long (split-path) spans at positions 63 mod 64
    and elsewhere: a slice whose last record is a skipped long span must still
    store its other results (large batches, where a slice holds up to 64
    records).  uniform: every span one task (runs of 64 records, no slice
    starts); else 32-task spans too (task-balanced slices)."""
    rng = np.random.default_rng(0x5EED0011)
    size = 48 << 20
    host = oracle.synth(size, 0x5EED0011)
    n = 300_000
    lens = rng.integers(0, 300, size=n).astype(np.uint64)
    idx_long = np.concatenate([np.arange(63, n, 64 * 37), rng.integers(0, n, size=200)])
    lens[idx_long] = rng.integers(131073, 400_000, size=len(idx_long))
    if not uniform:
        lens[rng.integers(0, n, size=500)] = 131072  # the longest span the span pass folds itself
    off = rng.integers(0, size - 400_001, size=n).astype(np.uint64)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    _check_spans(dev, oracle, host, off, lens, init, mask=True)


def test_log_header_padding_skip(dev, oracle, route):
    """LOG_HEADER batches run the span kernel that skips chunk 0's padding
    rounds: short records paired with multi-chunk ones, empty and 1-3 byte
    records, random offsets; CRCs and the verify flags against the oracle
    (the stored crc sits 6 bytes before each span, db/log_reader.cc:246-257)."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED0013)
    size = 32 << 20
    host = oracle.synth(size, 0x5EED0013)
    n = 20_000
    lens = np.where(rng.random(n) < 0.8, rng.integers(0, 1100, size=n),
                    rng.integers(1100, 40_000, size=n)).astype(np.uint64)
    lens[:50] = np.arange(50)
    off = rng.integers(6, size - 40_001, size=n).astype(np.uint64)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    want, _ = oracle.batch(host, off, lens, init)
    # store the masked crc 6 bytes before half of the spans
    good = rng.random(n) < 0.5
    for i in np.nonzero(good)[0][:2000]:
        o = int(off[i]) - 6
        host[o:o + 4] = np.frombuffer(np.uint32(oracle.mask(int(want[i]))).tobytes(), dtype=np.uint8)
    want, _ = oracle.batch(host, off, lens, init)  # stores may land inside other spans
    stored = np.array([int.from_bytes(host[int(o) - 6:int(o) - 2].tobytes(), "little") for o in off], dtype=np.uint64)
    want_bad = np.array([oracle.unmask(int(s)) != int(w) for s, w in zip(stored, want)], dtype=np.uint8)
    buf = _to_dev(host, dev)
    d_off = _to_dev(off.astype(np.int64), dev)
    d_len = _to_dev(lens.astype(np.uint32).view(np.int32), dev)
    d_init = _to_dev(init.view(np.int32), dev)
    out, _ = crc32c.batch(buf, d_off, d_len, d_init, log_header=True)
    np.testing.assert_array_equal(_u32(out), want)
    out2, mm = crc32c.batch(buf, d_off, d_len, d_init, verify=True, log_header=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out2), want)
    np.testing.assert_array_equal(mm.cpu().numpy(), want_bad)
    assert want_bad.sum() < n  # some stored crcs match


@pytest.mark.parametrize("n", [1, 7, 640, 5000])
def test_slices_with_empty_slices(dev, oracle, n, route):
    """Small batches of multi-task spans: the slice size drops to 1-2 tasks, so
    a 32-task span opens many empty slices that streams must step over."""
    rng = np.random.default_rng(0x5EED0012 + n)
    size = 16 << 20
    host = oracle.synth(size, 0x5EED0012)
    lens = rng.choice([0, 1, 3, 4095, 4096, 4097, 65536, 131072, 200_000], size=n).astype(np.uint64)
    off = rng.integers(0, size - 200_001, size=n).astype(np.uint64)
    _check_spans(dev, oracle, host, off, lens)


def test_verify_sst_fixture(dev, golden, route):
    """ReadBlock verify semantics on the reference-built SST, clean and corrupted."""
    import torch
    from prismdb_amd import crc32c

    blocks = golden["sst"]["blocks"]
    off = torch.tensor([b["offset"] for b in blocks], dtype=torch.int64, device=dev)
    lens = torch.tensor([b["size"] + 1 for b in blocks], dtype=torch.int32, device=dev)
    raw = np.frombuffer(golden["sst_bytes"], dtype=np.uint8).copy()
    buf = _to_dev(raw, dev)
    out, mm = crc32c.batch(buf, off, lens, mask=True, verify=True)
    assert mm.sum().item() == 0
    assert crc32c.as_u32(out) == [b["masked_crc"] for b in blocks]
    for victim in (0, 7, len(blocks) - 1):
        bad = raw.copy()
        bad[blocks[victim]["offset"] + blocks[victim]["size"] // 2] ^= 0x80
        _, mm = crc32c.batch(_to_dev(bad, dev), off, lens, verify=True)
        assert mm.cpu().tolist() == [1 if i == victim else 0 for i in range(len(blocks))]
    # a flipped trailer byte is a mismatch too
    bad = raw.copy()
    bad[blocks[3]["offset"] + blocks[3]["size"] + 2] ^= 1
    _, mm = crc32c.batch(_to_dev(bad, dev), off, lens, verify=True)
    assert mm.cpu().tolist() == [1 if i == 3 else 0 for i in range(len(blocks))]


def test_verify_fixed_mode(dev, oracle):
    """Fixed-stride verify: trailers written as Mask(crc) after each span."""
    import torch
    from prismdb_amd import crc32c

    nblk, L, S = 4096, 3988, 3992
    host = oracle.synth(nblk * S + 8, 0x5EED000A)
    want = oracle.batch_fixed(host, S, L, nblk)
    for i in range(nblk):
        host[i * S + L:i * S + L + 4] = np.frombuffer(int(oracle.mask(int(want[i]))).to_bytes(4, "little"),
                                                      dtype=np.uint8)
    host[17 * S + 5] ^= 4
    buf = _to_dev(host, dev)
    _, mm = crc32c.batch_fixed(buf, S, L, nblk, verify=True)
    torch.cuda.synchronize()
    assert np.nonzero(mm.cpu().numpy())[0].tolist() == [17]


@pytest.mark.parametrize("stride,length,nblk", [(3992, 3988, 4096), (4096, 4092, 4096), (256, 252, 20000),
                                                (260, 256, 5000), (12, 8, 50000), (8, 4, 9000),
                                                (4096, 2048, 3000), (4100, 1000, 7000), (4096, 4092, (1 << 20) + 77)])
def test_verify_fixed_geometries(dev, oracle, stride, length, nblk, kernel_path):
    """ReadBlock verify over fixed-stride spans on both kernels: clean
    trailers, a flipped data byte, a flipped trailer byte, first/last spans
    damaged; non-zero init against the oracle's verify; CRC output too."""
    import torch
    from prismdb_amd import crc32c

    host = oracle.synth(nblk * stride + 8, 0x5EED0010 + length)
    off = np.arange(nblk, dtype=np.uint64) * stride
    lens = np.full(nblk, length, dtype=np.uint32)
    want, _ = oracle.batch(host, off, lens)
    tr = (((want >> 15) | (want << 17)) + np.uint32(0xA282EAD8)).astype("<u4").view(np.uint8).reshape(-1, 4)
    idx = (off.astype(np.int64)[:, None] + length + np.arange(4)[None, :]).reshape(-1)
    host[idx] = tr.reshape(-1)
    bad = sorted({0, nblk // 3, nblk // 2, nblk - 1})
    host[int(off[nblk // 3]) + length // 2] ^= 0x20          # data byte
    host[int(off[nblk // 2]) + length + 3] ^= 0x01           # trailer byte
    host[int(off[0])] ^= 0x80
    host[int(off[nblk - 1]) + length - 1] ^= 0x02
    buf = _to_dev(host, dev)
    out, mm = crc32c.batch_fixed(buf, stride, length, nblk, verify=True)
    torch.cuda.synchronize()
    assert np.nonzero(mm.cpu().numpy())[0].tolist() == bad
    want2, wmm = oracle.batch(host, off, lens, verify=True)
    np.testing.assert_array_equal(_u32(out), want2)
    np.testing.assert_array_equal(mm.cpu().numpy(), wmm)
    init = 0x31415926
    out3, mm3 = crc32c.batch_fixed(buf, stride, length, nblk, init=init, verify=True)
    want3, wmm3 = oracle.batch(host, off, lens, np.full(nblk, init, dtype=np.uint32), verify=True)
    np.testing.assert_array_equal(_u32(out3), want3)
    np.testing.assert_array_equal(mm3.cpu().numpy(), wmm3)
    del buf
    torch.cuda.empty_cache()


def test_full_size_config2_properties(dev, oracle):
    """BASELINE config 2 at full size (16 Mi x 4 KiB = 64 GiB): fixed-stride and
    descriptor paths agree on every block; 4096 sampled blocks (and the first
    and last) equal the oracle on host-regenerated bytes."""
    import torch
    from prismdb_amd import crc32c

    free, _ = torch.cuda.mem_get_info()
    nblk, L = 1 << 24, 4096
    if free < nblk * L + (2 << 30):
        pytest.skip("not enough device memory for the full-size case")
    buf = torch.empty(nblk * L, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, SEED)
    out, _ = crc32c.batch_fixed(buf, L, L, nblk)
    off = torch.arange(nblk, dtype=torch.int64, device=dev) * L
    lens = torch.full((nblk,), L, dtype=torch.int32, device=dev)
    out2, _ = crc32c.batch(buf, off, lens)
    assert torch.equal(out, out2)
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([[0, nblk - 1], rng.integers(0, nblk, 4096)]))
    got = _u32(out[torch.from_numpy(idx).to(dev)])
    for j, i in enumerate(idx.tolist()):
        blk = oracle.synth(L, SEED, i * L)
        assert got[j] == oracle.value(blk.tobytes()), i
    del buf, off, lens, out, out2
    torch.cuda.empty_cache()


@pytest.mark.parametrize("nblk,length", [((1 << 20) + 37, 4096), ((1 << 20) + 127, 4092), ((1 << 20) + 1, 2048)])
def test_fixed_full_runs_partial_tail(dev, oracle, nblk, length):
    """Batches big enough for the fixed kernel's full 64-span runs, with a
    partial last run: every block against the descriptor path, the last
    run-and-a-half plus random samples against the oracle."""
    import torch
    from prismdb_amd import crc32c

    L = 4096
    buf = torch.empty(nblk * L, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, SEED)
    out, _ = crc32c.batch_fixed(buf, L, length, nblk, init=0xABCDEF01, mask=True)
    off = torch.arange(nblk, dtype=torch.int64, device=dev) * L
    lens = torch.full((nblk,), length, dtype=torch.int32, device=dev)
    init = torch.full((nblk,), 0xABCDEF01 - (1 << 32), dtype=torch.int32, device=dev)
    out2, _ = crc32c.batch(buf, off, lens, init, mask=True)
    assert torch.equal(out, out2)
    rng = np.random.default_rng(2)
    idx = np.unique(np.concatenate([np.arange(nblk - 200, nblk), rng.integers(0, nblk, 512)]))
    got = _u32(out[torch.from_numpy(idx).to(dev)])
    for j, i in enumerate(idx.tolist()):
        host = oracle.synth(length, SEED, i * L)
        want = oracle.batch_fixed(host, length, length, 1, init=0xABCDEF01, mask=True)[0]
        assert got[j] == want, i
    del buf, off, lens, init, out, out2
    torch.cuda.empty_cache()


def test_concurrent_streams(dev, oracle):
    """Two streams in flight at once give the same answers as one."""
    import torch
    from prismdb_amd import crc32c

    nblk, L = 8192, 4096
    buf = torch.empty(nblk * L, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, SEED)
    want = oracle.batch_fixed(buf.cpu().numpy(), L, L, nblk)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for s in (s1, s2, s1, s2):
        with torch.cuda.stream(s):
            o, _ = crc32c.batch_fixed(buf, L, L, nblk)
            off = torch.arange(nblk, dtype=torch.int64, device=dev) * L
            lens = torch.full((nblk,), L, dtype=torch.int32, device=dev)
            o2, _ = crc32c.batch(buf, off, lens)
            outs += [o, o2]
    torch.cuda.synchronize()
    for o in outs:
        assert (_u32(o) == want).all()


def test_concurrent_host_threads(dev, oracle):
    """Four host threads, each with its own stream, call the generic and the
    fixed path at once (ctypes drops the GIL): the per-(thread, device, stream)
    workspaces and the lock-free calls give every thread the oracle's answers."""
    import threading

    import torch
    from prismdb_amd import crc32c

    nblk, L = 4096, 4096
    buf = torch.empty(nblk * L + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0014)
    host = buf.cpu().numpy()
    rng = np.random.default_rng(0x5EED0014)
    jobs = []
    for t in range(4):
        n = 3000 + 500 * t
        lens = rng.integers(0, 40_000, size=n).astype(np.uint64)
        off = rng.integers(0, nblk * L - 40_001, size=n).astype(np.uint64)
        want, _ = oracle.batch(host, off, lens)
        jobs.append((off, lens, want))
    want_fixed = oracle.batch_fixed(host, L, L, nblk)
    errors = []

    def run(t):
        try:
            s = torch.cuda.Stream()
            off, lens, want = jobs[t]
            with torch.cuda.stream(s):
                d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
                d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
                for _ in range(5):
                    out, _ = crc32c.batch(buf, d_off, d_len)
                    outf, _ = crc32c.batch_fixed(buf, L, L, nblk)
                    s.synchronize()
                    if not (_u32(out) == want).all() or not (_u32(outf) == want_fixed).all():
                        errors.append(t)
                        return
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    assert not errors, errors


def test_host_resident_pipeline(dev, oracle):
    """leveldb_crc32c_batch_host: SST-shaped spans in pageable host memory and
    in a pinned buffer, > 64 MiB so several chunks are in flight; verify mode."""
    import torch
    from prismdb_amd import crc32c

    n = 40000  # 3988-B spans at stride 3992: ~152 MiB, three 64 MiB chunks
    off = np.arange(n, dtype=np.uint64) * 3992
    lens = np.full(n, 3988, dtype=np.uint32)
    host = oracle.synth(n * 3992 + 8, 0x5EED000C)
    want, _ = oracle.batch(host, off, lens)
    got, _ = crc32c.batch_host(host, off, lens)
    np.testing.assert_array_equal(got, want)
    pinned = torch.from_numpy(host).pin_memory()
    init = (np.arange(n, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    wantm, _ = oracle.batch(host, off, lens, init, mask=True)
    gotm, _ = crc32c.batch_host(pinned, off, lens, init, mask=True)
    np.testing.assert_array_equal(gotm, wantm)
    # verify: write Mask(crc) trailers after every span, break one
    for i in range(n):
        host[i * 3992 + 3988:i * 3992 + 3992] = np.frombuffer(
            int(oracle.mask(int(want[i]))).to_bytes(4, "little"), dtype=np.uint8)
    host[12345 * 3992 + 7] ^= 1
    _, mm = crc32c.batch_host(host, off, lens, verify=True)
    assert np.nonzero(mm)[0].tolist() == [12345]


@pytest.fixture(params=[32, 64])
def pipe_chunk(request):
    """The host pipeline's chunk size (tuning hook; 64 MiB by default)."""
    import ctypes

    from prismdb_amd import _lib

    L = _lib.lib()
    L.prismdb_pipeline_chunk_bytes.restype = ctypes.c_size_t
    L.prismdb_pipeline_chunk_bytes.argtypes = [ctypes.c_size_t]
    prev = L.prismdb_pipeline_chunk_bytes(request.param << 20)
    yield request.param
    L.prismdb_pipeline_chunk_bytes(prev)


def test_host_pipeline_mixed_large_spans(dev, oracle, pipe_chunk):
    """Host batches whose spans straddle the DMA chunk size (32 and 64 MiB):
    small spans, a 48 MiB span, a 64 MiB - 4 span verified with its trailer,
    then small spans again; with per-span init."""
    from prismdb_amd import crc32c

    lens = [3988] * 300 + [48 << 20, 1000, (64 << 20) - 4] + [4096] * 300 + [7, 0, 1]
    off, pos = [], 16
    for ln in lens:
        off.append(pos)
        pos += ln + 4 + (pos % 7)
    host = oracle.synth(pos + 64, 0x5EED000E)
    off = np.asarray(off, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint32)
    init = (np.arange(len(lens), dtype=np.uint64) * 0x9E3779B1 % (1 << 32)).astype(np.uint32)
    want, _ = oracle.batch(host, off, lens, init)
    got, _ = crc32c.batch_host(host, off, lens, init)
    np.testing.assert_array_equal(got, want)
    plain, _ = oracle.batch(host, off, lens)
    for i in range(len(lens)):
        o = int(off[i]) + int(lens[i])
        host[o:o + 4] = np.frombuffer(int(oracle.mask(int(plain[i]))).to_bytes(4, "little"), dtype=np.uint8)
    host[int(off[302]) + 12345678] ^= 0x10
    _, mm = crc32c.batch_host(host, off, lens, verify=True)
    assert np.nonzero(mm)[0].tolist() == [302]


def _sealed_image(oracle, host, off, lens, log_header=False):
    """The oracle's sealed copy of `host`: every span's Mask(Value(span))
    stored as 4 LE bytes after it (TableBuilder::WriteRawBlock,
    table/table_builder.cc:192-197) or, for log records, 6 bytes before it
    (log::Writer::EmitPhysicalRecord, db/log_writer.cc:90-97)."""
    want = host.copy()
    crc, _ = oracle.batch(host, off, lens, mask=True)
    at = (off.astype(np.int64) - 6) if log_header else (off.astype(np.int64) + lens.astype(np.int64))
    want[at[:, None] + np.arange(4)[None, :]] = crc.astype("<u4").view(np.uint8).reshape(-1, 4)
    return want, crc


@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline_seal_trailers(dev, oracle, pinned):
    """leveldb_crc32c_batch_host with WRITE_TRAILER: a 152 MiB SST-shaped
    image (3988-B contents||type spans at stride 3992, three 64 MiB chunks)
    with zeroed trailers, pageable and pinned: afterwards every byte of the
    buffer equals the oracle-sealed image, and the returned crcs are the
    masked values; a verify pass over the result flags nothing."""
    import torch
    from prismdb_amd import crc32c

    n = 40000
    off = np.arange(n, dtype=np.uint64) * 3992
    lens = np.full(n, 3988, dtype=np.uint32)
    img = oracle.synth(n * 3992 + 8, 0x5EED0013)
    img[(off + 3988).astype(np.int64)[:, None] + np.arange(4)[None, :]] = 0
    want, crc = _sealed_image(oracle, img, off, lens)
    host = torch.from_numpy(img.copy()).pin_memory() if pinned else img.copy()
    got, _ = crc32c.batch_host(host, off, lens, mask=True, trailer=True)
    np.testing.assert_array_equal(got, crc)
    after = host.numpy() if pinned else host
    assert (after == want).all(), np.nonzero(after != want)[0][:8]
    _, mm = crc32c.batch_host(host, off, lens, verify=True)
    assert int(mm.sum()) == 0


def test_host_pipeline_seal_log_headers(dev, oracle, pipe_chunk32):
    """WRITE_TRAILER | LOG_HEADER on the host path: log records of 0..1280
    payload bytes (span = type||payload) at odd offsets over several 32 MiB
    chunks; the header crc 6 bytes before each span is written and nothing
    else changes."""
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED0014)
    lens = rng.integers(1, 1282, size=60000).astype(np.uint32)
    off = np.empty(len(lens), dtype=np.uint64)
    pos = 13
    for i, ln in enumerate(lens):
        off[i] = pos + 6  # crc[4] length[2] | type||payload
        pos += 6 + int(ln) + int(rng.integers(0, 9))
    img = oracle.synth(pos + 16, 0x5EED0015)
    want, crc = _sealed_image(oracle, img, off, lens, log_header=True)
    host = img.copy()
    got, _ = crc32c.batch_host(host, off, lens, mask=True, trailer=True, log_header=True)
    np.testing.assert_array_equal(got, crc)
    assert (host == want).all(), np.nonzero(host != want)[0][:8]


def test_host_pipeline_seal_failure_drains(dev, oracle, pipe_chunk32):
    """A sealing host batch that fails after chunks are in flight returns an
    error, writes no trailer past the chunks it finished, and the next sealing
    call (same ring) seals the whole image exactly."""
    import ctypes

    from prismdb_amd import _lib, crc32c

    L = _lib.lib()
    L.prismdb_pipeline_fail_after.argtypes = [ctypes.c_int]
    n = 40000
    off = np.arange(n, dtype=np.uint64) * 3992
    lens = np.full(n, 3988, dtype=np.uint32)
    img = oracle.synth(n * 3992 + 8, 0x5EED0016)
    tr = (off + 3988).astype(np.int64)[:, None] + np.arange(4)[None, :]
    img[tr] = 0
    want, _ = _sealed_image(oracle, img, off, lens)
    host = img.copy()
    L.prismdb_pipeline_fail_after(3)
    try:
        with pytest.raises(RuntimeError, match="injected failure"):
            crc32c.batch_host(host, off, lens, mask=True, trailer=True)
    finally:
        L.prismdb_pipeline_fail_after(0)
    # spans outside the trailers never change; trailers are either still zero
    # or already their sealed value (chunks finished before the failure)
    body = np.ones(host.size, dtype=bool)
    body[tr.reshape(-1)] = False
    assert (host[body] == img[body]).all()
    t_got, t_want = host[tr], want[tr]
    assert ((t_got == 0).all(axis=1) | (t_got == t_want).all(axis=1)).all()
    crc32c.batch_host(host, off, lens, mask=True, trailer=True)
    assert (host == want).all()


@pytest.fixture
def pipe_chunk32():
    """32 MiB host pipeline chunks for the test (the default is 64 MiB)."""
    import ctypes

    from prismdb_amd import _lib

    L = _lib.lib()
    L.prismdb_pipeline_chunk_bytes.restype = ctypes.c_size_t
    L.prismdb_pipeline_chunk_bytes.argtypes = [ctypes.c_size_t]
    prev = L.prismdb_pipeline_chunk_bytes(32 << 20)
    yield 32
    L.prismdb_pipeline_chunk_bytes(prev)


def test_host_pipeline_failure_drains_ring(dev, oracle, pipe_chunk32):
    """A host batch that fails after several chunks are in flight returns its
    ring to the pool empty: the next, smaller call (which leases it again)
    gets its own results only and nothing is written past its output arrays."""
    import ctypes

    from prismdb_amd import _lib, crc32c

    L = _lib.lib()
    L.prismdb_pipeline_fail_after.argtypes = [ctypes.c_int]
    n = 40000  # ~152 MiB at stride 3992: five 32 MiB chunks (pipe_chunk32), three in flight at the failure
    off = np.arange(n, dtype=np.uint64) * 3992
    lens = np.full(n, 3988, dtype=np.uint32)
    host = oracle.synth(n * 3992 + 8, 0x5EED0010)
    L.prismdb_pipeline_fail_after(3)
    try:
        with pytest.raises(RuntimeError, match="injected failure"):
            crc32c.batch_host(host, off, lens, verify=True)
    finally:
        L.prismdb_pipeline_fail_after(0)
    m, guard = 100, 4096
    out = np.full(m + guard, 0xA5A5A5A5, dtype=np.uint32)
    mm = np.full(m + guard, 0x5A, dtype=np.uint8)
    rc = L.leveldb_crc32c_batch_host(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(off.ctypes.data),
                                     ctypes.c_void_p(lens.ctypes.data), None, ctypes.c_size_t(m),
                                     ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(mm.ctypes.data),
                                     ctypes.c_uint32(0))
    assert rc == 0, L.leveldb_crc32c_last_error()
    want, _ = oracle.batch(host, off[:m], lens[:m])
    np.testing.assert_array_equal(out[:m], want)
    assert (out[m:] == 0xA5A5A5A5).all() and (mm[m:] == 0x5A).all()
    # and a full call afterwards is whole again
    got, _ = crc32c.batch_host(host, off, lens)
    want, _ = oracle.batch(host, off, lens)
    np.testing.assert_array_equal(got, want)


def test_host_pipeline_many_threads(dev, oracle):
    """Host batches from 6 threads at once, then from 24 short-lived threads
    (rings leased from the per-device pool, more concurrent calls than idle
    rings kept): every call bit-exact, verify and mask mixed."""
    import threading

    from prismdb_amd import crc32c

    n = 12000  # ~46 MiB: two chunks
    off = np.arange(n, dtype=np.uint64) * 3992
    lens = np.full(n, 3988, dtype=np.uint32)
    host = oracle.synth(n * 3992 + 8, 0x5EED0011)
    raw, _ = oracle.batch(host, off, lens)
    masked, _ = oracle.batch(host, off, lens, mask=True)
    errors = []

    def run(t):
        try:
            got, _ = crc32c.batch_host(host, off, lens, mask=bool(t & 1))
            if not (got == (masked if t & 1 else raw)).all():
                errors.append(t)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    for first, count in ((0, 6), (6, 8), (14, 8), (22, 8)):
        th = [threading.Thread(target=run, args=(first + t,)) for t in range(count)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
    assert not errors, errors


def test_host_pipeline_ring_workspaces_released(dev, oracle):
    """A long-lived thread (this one) calling batch_host next to 7 others,
    three times: every call leases a ring (8 at once; the pool keeps 2 idle
    and frees the rest), and the batch workspace of a ring's stream goes
    with the ring -- it used to stay in each calling thread's cache (up to 8
    per thread, ~70 MB each), so this thread's device memory grew.  Device
    memory after the rounds is within 200 MB of before."""
    import threading

    import torch
    from prismdb_amd import crc32c

    n = 12000
    off = np.arange(n, dtype=np.uint64) * 3992
    lens = np.full(n, 3988, dtype=np.uint32)
    host = oracle.synth(n * 3992 + 8, 0x5EED0012)
    raw, _ = oracle.batch(host, off, lens)
    errors = []

    def run(t):
        try:
            got, _ = crc32c.batch_host(host, off, lens)
            if not (got == raw).all():
                errors.append(t)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    def round_(k):
        th = [threading.Thread(target=run, args=(t,)) for t in range(k - 1)]
        for x in th:
            x.start()
        run(-1)  # this thread too
        for x in th:
            x.join(120)

    round_(2)  # two rings idle in the pool from here on
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(dev)
    for _ in range(3):
        round_(8)
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(dev)
    assert not errors, errors
    assert free0 - free1 < 200 << 20, (free0 - free1) / 2**20


@pytest.fixture(params=["lane_all", "direct"])
def short_route(request, native):
    """Short records through the lane kernel (every planner batch) and through
    the one-launch kernel."""
    from conftest import set_route

    restore = set_route(native, request.param)
    yield request.param
    restore()


@pytest.mark.parametrize("log_header", [False, True])
def test_short_records(dev, oracle, short_route, log_header):
    """Short records on every length 0..1280 at every alignment, the lengths
    just above the lane kernel's limit (its generic path), random init, verify
    with the stored crc after the span or (log records) 6 bytes before it, one
    damaged record in four; record counts that end mid-run."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED0020 + log_header)
    lens = np.concatenate([np.arange(0, 1281), [1281, 1282, 1283, 1284, 2000, 4096, 5000, 70_000],
                           rng.integers(0, 1281, size=3000)]).astype(np.uint64)
    rng.shuffle(lens)
    n = len(lens) - 3  # 4290: not a multiple of 4 or of 64
    lens = lens[:n]
    gaps = rng.integers(6, 30, size=n).astype(np.uint64)
    off = np.cumsum(np.concatenate([[7], (lens + gaps)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 64, 0x5EED0021)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    raw, _ = oracle.batch(host, off, lens, init)
    pos = off.astype(np.int64) - 6 if log_header else (off + lens).astype(np.int64)
    damaged = rng.random(n) < 0.25
    for i in range(n):
        c = oracle.mask(int(raw[i])) ^ (1 if damaged[i] else 0)
        host[pos[i]:pos[i] + 4] = np.frombuffer(np.uint32(c).tobytes(), dtype=np.uint8)
    want, _ = oracle.batch(host, off, lens, init, mask=True)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev)
    out, mm = crc32c.batch(buf, d_off, d_len, d_init, mask=True, verify=True, log_header=log_header)
    np.testing.assert_array_equal(_u32(out), want)
    np.testing.assert_array_equal(mm.cpu().numpy(), damaged.astype(np.uint8))
    out2, _ = crc32c.batch(buf, d_off, d_len)  # no init, no mask, no verify
    np.testing.assert_array_equal(_u32(out2), oracle.batch(host, off, lens)[0])


def test_short_records_far_apart(dev, oracle, short_route):
    """Neighbouring records more than 2 GiB apart (64-bit addresses in the
    lane kernel's runs and the one-launch kernel's static runs)."""
    import torch
    from prismdb_amd import crc32c

    far = (2 << 30) + (256 << 20)
    buf = torch.empty(far + (4 << 20), dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf[:4 << 20], 0x5EED0022)
    crc32c.fill_synthetic(buf[far:], 0x5EED0023)
    lo = buf[:4 << 20].cpu().numpy()
    hi = buf[far:].cpu().numpy()
    rng = np.random.default_rng(0x5EED0024)
    n = 1000
    lens = rng.integers(0, 1281, size=n).astype(np.uint64)
    rel = rng.integers(8, (4 << 20) - 1300, size=n).astype(np.uint64)
    side = rng.random(n) < 0.4  # in the far region
    off = rel + np.where(side, np.uint64(far), np.uint64(0))
    want = np.empty(n, dtype=np.uint32)
    for region, sel in ((lo, ~side), (hi, side)):
        want[sel] = oracle.batch(region, rel[sel], lens[sel])[0]
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    out, _ = crc32c.batch(buf, d_off, d_len)
    np.testing.assert_array_equal(_u32(out), want)
    del buf
    torch.cuda.empty_cache()


def test_lane_claimed_tail_runs(dev, oracle, native):
    """A log-record batch large enough for the lane kernel's claimed tail
    (more than (kLaneTailRounds + 2) runs of 64 records per wave: its last
    rounds of runs are claimed from a per-call counter): 1.6 M short records
    with a few long ones among them (the generic path), every record's
    result bit-exact and every damaged one flagged."""
    import torch
    from conftest import set_route
    from prismdb_amd import crc32c

    import torch as _t

    rng = np.random.default_rng(0x5EED0070)
    cus = _t.cuda.get_device_properties(0).multi_processor_count
    n = max(1_600_000, 64 * 11 * 8 * cus)  # > (kLaneTailRounds + 2) runs per wave (8 waves per CU)
    lens = rng.integers(8, 200, size=n).astype(np.uint64)
    lens[rng.integers(0, n, size=300)] = rng.integers(1281, 4000, size=300).astype(np.uint64)
    gaps = rng.integers(7, 20, size=n).astype(np.uint64)
    off = np.cumsum(np.concatenate([[11], (lens + gaps)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 64, 0x5EED0071)
    raw, _ = oracle.batch(host, off, lens)
    damaged = rng.random(n) < 0.01
    masked = ((raw.astype(np.uint64) << np.uint64(17) | raw.astype(np.uint64) >> np.uint64(15)) & np.uint64(0xFFFFFFFF))
    masked = ((masked + np.uint64(0xa282ead8)) & np.uint64(0xFFFFFFFF)).astype(np.uint32) ^ damaged.astype(np.uint32)
    pos = off.astype(np.int64) - 6
    view = host[:int(pos[-1]) + 4 + 64]
    idx = pos[:, None] + np.arange(4)[None, :]
    view[idx] = masked.view(np.uint8).reshape(-1, 4)
    want, _ = oracle.batch(host, off, lens, mask=True)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    restore = set_route(native, "lane_log")
    try:
        out, mm = crc32c.batch(buf, d_off, d_len, mask=True, verify=True, log_header=True)
        claims = _last_claims(native)
    finally:
        restore()
    np.testing.assert_array_equal(_u32(out), want)
    np.testing.assert_array_equal(mm.cpu().numpy(), damaged.astype(np.uint8))
    assert oracle.mask(int(raw[0])) == int(masked[0] ^ damaged[0])
    assert claims[1] > 0, "the lane kernel's tail was never claimed"


def _last_claims(native):
    """{span / pair-run kernel claims, lane kernel claims} of this thread's
    last planner-path batch (test hook prismdb_crc32c_last_claims)."""
    arr = (ctypes.c_uint64 * 2)()
    assert native.prismdb_crc32c_last_claims(arr) == 0
    return list(arr)


@pytest.mark.parametrize("kernel", ["pair", "pair_short", "span"])
def test_claimed_tails_engage(dev, oracle, native, kernel):
    """Batches sized from the device's CU count so that the planner kernels'
    claimed tails engage: the pair-run kernel (one-task spans: 64 B spans,
    ~2300 per wave, ~18 pairs per run; pair_short: ~600 per wave, ~4.7 pairs
    per run, config 5's shape, whose claims ride one run ahead on the eight
    claim counters) and the span kernel (task-balanced slices of >= 32
    tasks, 16 per stream: spans of 1-3 chunks, ~16 GiB).  The claims read
    back are > 0, and the results are bit-exact: every span for the pair
    batches, a sample plus the ends (host-regenerated bytes) for the span
    batch."""
    import torch
    from prismdb_amd import crc32c

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nwaves = 16 * cus  # kWavesPerGroup, one group per CU
    seed = 0x5EED0080 + (kernel == "span") + 2 * (kernel == "pair_short")
    if kernel in ("pair", "pair_short"):
        n = (2300 if kernel == "pair" else 600) * nwaves  # np / (64 nwaves): ~18 / ~4.7 pairs per run
        off = np.arange(n, dtype=np.uint64) * 64 + 3
        lens = np.full(n, 61, dtype=np.uint32)
        host = oracle.synth(n * 64 + 64, seed)
        buf = torch.from_numpy(host).to(dev)
    else:
        rng = np.random.default_rng(seed)
        streams = 2 * nwaves
        tasks_per_span = rng.integers(1, 4, size=int(600 * streams / 2)).astype(np.uint64)  # ~600 tasks per stream
        lens = (tasks_per_span * 4096 - rng.integers(0, 300, size=len(tasks_per_span)).astype(np.uint64)).astype(np.uint32)
        n = len(lens)
        off = np.cumsum(np.concatenate([[5], lens[:-1].astype(np.uint64) + 7])).astype(np.uint64)
        total = int(off[-1]) + int(lens[-1]) + 64
        free, _ = torch.cuda.mem_get_info()
        if free < total + (4 << 30):
            pytest.skip("not enough device memory")
        buf = torch.empty(total, dtype=torch.uint8, device=dev)
        crc32c.fill_synthetic(buf, seed)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    restore = set_route_planner(native)
    try:
        out, _ = crc32c.batch(buf, d_off, d_len, mask=True, check_bounds=False)
        sched = (ctypes.c_uint64 * 3)()
        assert native.prismdb_crc32c_last_schedule(sched) == 0
        claims = _last_claims(native)
    finally:
        restore()
    got = _u32(out)
    if kernel != "span":
        assert sched[1] == 0 and sched[2] == 1  # every record one task: the pair-run kernel's schedule
        want, _ = oracle.batch(host, off, lens, mask=True)
        np.testing.assert_array_equal(got, want)
    else:
        assert sched[1] > 0 and sched[0] // sched[1] >= 32, list(sched)  # task-balanced slices of >= 32 tasks
        idx = np.unique(np.concatenate([[0, n - 1], np.random.default_rng(1).integers(0, n, 2048)]))
        for i in idx.tolist():
            blk = oracle.synth(int(lens[i]), seed, int(off[i]))
            assert int(got[i]) == oracle.mask(oracle.value(blk.tobytes())), i
    assert claims[0] > 0, f"the {kernel} kernel's tail was never claimed ({list(sched)})"
    del buf, d_off, d_len, out
    torch.cuda.empty_cache()


def set_route_planner(native):
    from conftest import set_route

    return set_route(native, "span_only")


@pytest.mark.parametrize("layout", ["runs", "all_long", "one_short_run", "under_a_run"])
def test_lane_runs_without_owned_records(dev, oracle, native, layout):
    """Log-record batches on the lane route whose runs of 64 spans hold no
    record the lane kernel owns (all > 1280 B): the lane kernel visits every
    run (it no longer skips them by a flag) and reads the zero region there,
    while the long-span list -- built on the side stream next to it -- sends
    those records through the generic path.  Whole long runs, whole short
    runs and mixed ones; a batch of long records only; one short run among
    long ones; fewer spans than a run.  Bit-exact, verify flags included."""
    import torch
    from conftest import set_route
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED0060)
    kinds = {"runs": ["L"] * 64 + ["S"] * 64 + ["L"] * 30 + ["S"] * 34 + ["L"] * 128 + ["S"] * 17,
             "all_long": ["L"] * 200,
             "one_short_run": ["L"] * 192 + ["S"] * 64 + ["L"] * 64,
             "under_a_run": ["L"] * 20 + ["S"] * 9}[layout]
    lens = np.array([rng.integers(1281, 9000) if k == "L" else rng.integers(8, 1281) for k in kinds], dtype=np.uint64)
    n = len(lens)
    gaps = rng.integers(7, 40, size=n).astype(np.uint64)
    off = np.cumsum(np.concatenate([[13], (lens + gaps)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 64, 0x5EED0061)
    raw, _ = oracle.batch(host, off, lens)
    damaged = rng.random(n) < 0.2
    for i in range(n):  # stored crc 6 B before each span (log::Writer's header)
        c = oracle.mask(int(raw[i])) ^ (2 if damaged[i] else 0)
        host[int(off[i]) - 6:int(off[i]) - 2] = np.frombuffer(np.uint32(c).tobytes(), dtype=np.uint8)
    want, _ = oracle.batch(host, off, lens, mask=True)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    restore = set_route(native, "lane_log")
    try:
        out, mm = crc32c.batch(buf, d_off, d_len, mask=True, verify=True, log_header=True)
        listed = _last_split(native)[3]
    finally:
        restore()
    np.testing.assert_array_equal(_u32(out), want)
    np.testing.assert_array_equal(mm.cpu().numpy(), damaged.astype(np.uint8))
    assert listed == kinds.count("L")
    """One caller stream, three planner-path batches in a row reusing one
    workspace: spans that are not log records, then the same spans as log
    records (the lane kernel and its list in front), then the first batch
    again.  Round 4 once planned the first kind for half the span-kernel
    streams, and the second laid its slice starts out past the block the
    first had sized (an illegal address in smoke()): the workspace now
    follows the largest stream count it served.  Every result against the
    oracle."""
    import torch
    from prismdb_amd import crc32c
    from conftest import set_route

    rng = np.random.default_rng(0x5EED0090)
    n = 3000
    lens = rng.integers(1, 1200, size=n).astype(np.uint32)
    off = (np.cumsum(lens.astype(np.uint64) + 11) - lens.astype(np.uint64) + 7).astype(np.uint64)
    host = oracle.synth(int(off[-1]) + int(lens[-1]) + 64, 0x5EED0091)
    want, _ = oracle.batch(host, off, lens)
    s = torch.cuda.Stream(dev)
    restore = set_route(native, "lane_log")  # the planner path for every size
    try:
        with torch.cuda.stream(s):
            buf = torch.from_numpy(host).to(dev)
            d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
            d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        outs = []
        for log_header in (False, True, False):
            o, _ = crc32c.batch(buf, d_off, d_len, log_header=log_header, stream=s, check_bounds=False)
            outs.append(o)
        s.synchronize()
    finally:
        restore()
    for o in outs:
        np.testing.assert_array_equal(_u32(o), want)


def test_band_routing_by_caller_intent(dev, oracle, native):
    """2^17 < n <= 2^18 spans with the default routing: a plain checksum batch
    takes the planner path, the same spans sealed or verified take the
    one-launch kernel (one launch up to its 196 608-span capacity, as these
    150 000; two windows above: include/prismdb_crc32c.h); bit-exact on every
    route."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED0090)
    n = 150_000
    lens = rng.choice([100, 1000, 3000, 9000], size=n).astype(np.uint64)
    off = np.cumsum(np.concatenate([[8], (lens + 4)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 64, 0x5EED0091)
    raw, _ = oracle.batch(host, off, lens)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    assert native.prismdb_crc32c_windows(2) == 2 and native.prismdb_crc32c_direct_max(1 << 17) == 1 << 17
    sched = (ctypes.c_uint64 * 3)()
    out, _ = crc32c.batch(buf, d_off, d_len)
    assert native.prismdb_crc32c_last_schedule(sched) == 0  # the planner path
    np.testing.assert_array_equal(_u32(out), raw)
    out, _ = crc32c.batch(buf, d_off, d_len, mask=True, trailer=True)
    assert native.prismdb_crc32c_last_schedule(sched) == -2  # the one-launch kernel
    masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    np.testing.assert_array_equal(_u32(out), masked)
    out, mm = crc32c.batch(buf, d_off, d_len, verify=True)
    assert native.prismdb_crc32c_last_schedule(sched) == -2
    np.testing.assert_array_equal(_u32(out), raw)
    assert not mm.cpu().numpy().any()


def test_pair_tail_claims_repeat_against_fixed_kernel(dev):
    """Config 5's data blocks (2.4 M spans of 3988 B at stride 3992: the
    pair-run kernel, ~4.7 pairs per run, its tail claimed one run ahead on
    eight counters) ten times over: the claims deal the tail runs in a
    different order every call, and every call's results equal the fixed
    kernel's over the same blocks (an independent kernel; tools/claim_stress.py
    runs the same at 60 calls plus sealed config-5 partitions)."""
    import torch
    from prismdb_amd import crc32c

    n = 2404116
    free, _ = torch.cuda.mem_get_info()
    if free < n * 3992 + (2 << 30):
        pytest.skip("not enough device memory")
    buf = torch.empty(n * 3992 + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0C5C)
    want, _ = crc32c.batch_fixed(buf, 3992, 3988, n, mask=True)
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * 3992
    d_len = torch.full((n,), 3988, dtype=torch.int32, device=dev)
    for _ in range(10):
        out, _ = crc32c.batch(buf, d_off, d_len, mask=True, check_bounds=False)
        assert int((out != want).sum().item()) == 0
    del buf, d_off, d_len, want, out
    torch.cuda.empty_cache()
