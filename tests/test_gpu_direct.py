"""The one-launch descriptor path (prismdb_amd/csrc/crc32c_direct.hip) at the
granularity PrismDB calls at: one SST file per call (TableBuilder::Finish,
table/table_builder.cc:185-261; ReadBlock verify over a compaction input,
table/format.cc:91-102), many calls back to back on one stream; and its
machinery: tickets of long spans claimed by any wave, the combine, the
whole-span fallback when the ticket workspace is full, orphaned claims
adopted by a late pusher.  Bit-exact against the oracle."""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ND, DATA, STRIDE, INDEX = 16811, 3988, 3992, 486977  # one 64 MiB-class SST


@pytest.fixture(scope="module")
def dev(native):
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    from prismdb_amd import crc32c

    crc32c.device_init(0)
    return torch.device("cuda", 0)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _stats(native):
    arr = (ctypes.c_uint64 * 4)()
    assert native.prismdb_crc32c_direct_stats(arr) == 0
    return np.array(arr, dtype=np.int64)


def _last_split_rc(native):
    arr = (ctypes.c_uint64 * 4)()
    return native.prismdb_crc32c_last_split(arr)


def _sst_file(oracle, seed, files=1):
    """`files` SST-shaped files back to back: per file 16 811 data spans
    (contents || type, 3988 B at stride 3992) and the index span, each with
    its masked crc stored after it (a sealed file).  Returns host bytes,
    offsets, lengths and the masked crcs."""
    fbytes = ND * STRIDE + INDEX + 4
    off1 = np.concatenate([np.arange(ND, dtype=np.uint64) * STRIDE, np.array([ND * STRIDE], dtype=np.uint64)])
    len1 = np.concatenate([np.full(ND, DATA, dtype=np.uint32), np.array([INDEX], dtype=np.uint32)])
    host = oracle.synth(files * fbytes + 64, seed)
    off = (np.arange(files, dtype=np.uint64)[:, None] * fbytes + off1[None, :]).reshape(-1) + 8
    lens = np.tile(len1, files)
    raw, _ = oracle.batch(host, off, lens)
    masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    tr = (off + lens.astype(np.uint64)).astype(np.int64)[:, None] + np.arange(4)[None, :]
    host[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
    return host, off, lens, raw, masked


def test_sst_file_calls_back_to_back(dev, oracle, native):
    """100 single-file calls enqueued back to back on one stream, alternating
    WriteRawBlock sealing (MASK | WRITE_TRAILER: rewrites the same trailers)
    and ReadBlock verify, each into its own result arrays; every result of
    every call against the oracle.  The calls take the one-launch path."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00D1)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    n = len(off)
    calls = 100
    outs = torch.empty((calls, n), dtype=torch.int32, device=dev)
    mms = torch.full((calls, n), 7, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for i in range(calls):
        if i % 2 == 0:
            crc32c.batch(buf, d_off, d_len, mask=True, trailer=True, out=outs[i], check_bounds=False)
        else:
            crc32c.batch(buf, d_off, d_len, verify=True, out=outs[i], mismatch=mms[i], check_bounds=False)
    torch.cuda.synchronize()
    assert _last_split_rc(native) == -2  # the one-launch path
    got = outs.cpu().numpy().view(np.uint32)
    for i in range(calls):
        np.testing.assert_array_equal(got[i], masked if i % 2 == 0 else raw, err_msg=f"call {i}")
    mm = mms.cpu().numpy()
    assert (mm[1::2] == 0).all()
    assert (buf.cpu().numpy() == host).all()  # the trailers written equal the stored ones


@pytest.mark.parametrize("files", [1, 7])
def test_sst_files_verify_damaged(dev, oracle, native, files):
    """Verify one and seven files per call (7 x 16 812 spans: the one-launch
    limit is 2^17) with damaged data blocks, a damaged index block (its
    tickets) and a damaged trailer; then a non-zero init on every span."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00D2 + files, files)
    n = len(off)
    victims = [3, n - 1, (n // 2) | 1, ND]  # data blocks, the last file's index, the first file's index
    for v in victims[:3]:
        host[int(off[v]) + int(lens[v]) // 3] ^= 0x11
    host[int(off[victims[3]]) + int(lens[victims[3]]) + 1] ^= 0x80  # trailer byte
    want, wmm = oracle.batch(host, off, lens, verify=True)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    out, mm = crc32c.batch(buf, d_off, d_len, verify=True)
    assert _last_split_rc(native) == -2
    np.testing.assert_array_equal(_u32(out), want)
    np.testing.assert_array_equal(mm.cpu().numpy(), wmm)
    assert sorted(np.flatnonzero(mm.cpu().numpy()).tolist()) == sorted(set(victims))
    # a non-zero init on every span (Extend), masked
    init = (np.arange(n, dtype=np.uint64) * 0x9E3779B1 % (1 << 32)).astype(np.uint32)
    want2, _ = oracle.batch(host, off, lens, init, mask=True)
    out2, _ = crc32c.batch(buf, d_off, d_len, torch.from_numpy(init.view(np.int32)).to(dev), mask=True)
    np.testing.assert_array_equal(_u32(out2), want2)


@pytest.mark.parametrize("files", [1, 7])
def test_sst_files_seal_zeroed_trailers(dev, oracle, native, files):
    """WriteRawBlock over one and seven files per call into zeroed trailers
    (the ring spans' non-temporal trailer stores, the index block's through
    its tickets): every trailer is the masked crc again and no other byte of
    the buffer moves."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00D4 + files, files)
    n = len(off)
    tr = (off + lens.astype(np.uint64)).astype(np.int64)[:, None] + np.arange(4)[None, :]
    zeroed = host.copy()
    zeroed[tr] = 0
    buf = torch.from_numpy(zeroed).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    out, _ = crc32c.batch(buf, d_off, d_len, mask=True, trailer=True)
    assert _last_split_rc(native) == -2
    np.testing.assert_array_equal(_u32(out), masked)
    got = buf.cpu().numpy()
    np.testing.assert_array_equal(got[tr], host[tr])
    assert (got == host).all()
    assert n == files * (ND + 1)


RING_CHUNKS = 32  # kRingChunks: spans of up to 32 chunks of 4 KiB are folded in the static ring
TICKET_LG_MIN = 2  # kTicketLgMin


def nwaves():
    """The one-launch kernel's waves: 12 per CU."""
    import torch

    return 12 * torch.cuda.get_device_properties(0).multi_processor_count


def _ceil_lg(x):
    return 0 if x <= 1 else (x - 1).bit_length()


def ticket_lg(nch, n):
    """crc32c_direct.hip's ticket_lg: the smallest 2^lg >= 2^TICKET_LG_MIN
    chunks per ticket that keeps a span at <= 2^lt tickets, lt =
    floor(log2(2 nwaves)) - ceil(log2(n)) clamped to 6..12."""
    lt = min(12, max(6, (2 * nwaves()).bit_length() - 1 - _ceil_lg(n)))
    return max(_ceil_lg((nch + (1 << lt) - 1) >> lt), TICKET_LG_MIN)


def test_tickets_claimed_and_combined(dev, oracle, native):
    """Long spans (more than 32 chunks) of every ticket size from 4 to 256
    chunks (<= 64 tickets per span) mixed with short and ring-folded
    multi-chunk ones, at odd offsets, random init, MASK; the counters account
    for every ticket (claimed early, late or adopted) and no span was folded
    whole."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00D3)
    long_lens = [4097, 8192 + 5, 16 * 4096 + 3, 20 * 4096 + 11, 33 * 4096 + 9, 64 * 4096 - 5, 64 * 4096 + 1, 65 * 4096, 300_001,
                 1 << 20, (4 << 20) + 3, 2 * 4096 * 64 + 7, (32 << 20) + 1001, (64 << 20) - 3]
    lens = np.concatenate([rng.integers(0, 4097, size=3000), long_lens]).astype(np.uint64)
    rng.shuffle(lens)
    gaps = rng.integers(0, 9, size=len(lens)).astype(np.uint64)
    off = np.cumsum(np.concatenate([[5], (lens + gaps)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 16, 0x5EED00D4)
    init = rng.integers(0, 2**32, size=len(lens), dtype=np.uint64).astype(np.uint32)
    want, _ = oracle.batch(host, off, lens, init, mask=True)

    def tickets(L, o):
        h = (4 - (8 + o) % 4) % 4  # the device buffer starts 256-B aligned
        h = min(h, L)
        W = (L - h) // 4
        nch = (W + 1023) // 1024
        if nch <= RING_CHUNKS:
            return 0
        lg = ticket_lg(nch, len(lens))
        return (nch + (1 << lg) - 1) >> lg

    buf = torch.empty(len(host) + 8, dtype=torch.uint8, device=dev)
    buf[8:] = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy((off + 8).astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev)
    crc32c.batch(buf, d_off[:1], d_len[:1])  # this thread's workspace exists
    before = _stats(native)
    out, _ = crc32c.batch(buf, d_off, d_len, d_init, mask=True)
    after = _stats(native)
    np.testing.assert_array_equal(_u32(out), want)
    expect = sum(tickets(int(L), int(o)) for L, o in zip(lens, off))
    d = after - before
    assert d[1] == 0  # no span folded whole
    assert d[0] + d[2] + d[3] == expect, (d, expect)


@pytest.mark.parametrize("mode", ["plain", "verify", "seal", "log_verify"])
def test_ring_multichunk_spans(dev, oracle, native, mode):
    """Spans of 2..32 chunks are folded by their run's wave in the static
    ring, chunk after chunk on one stream (no tickets: the counters do not
    move).  Every chunk count at lengths around the chunk boundaries, every
    start alignment, random init, mixed with one-chunk spans; verify against
    a trailer (a few damaged), sealing (WRITE_TRAILER), and log-record verify
    (the stored crc 6 B before the span)."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00E1 + len(mode))
    lens = []
    for k in range(1, RING_CHUNKS + 1):
        for d in (-3, -1, 0, 1, 2, 5):
            L = k * 4096 + d
            if 0 < L <= RING_CHUNKS * 4096 - 4:  # body <= 32 chunks at any alignment
                lens.append(L)
    lens = np.array(lens + rng.integers(0, 4097, size=400).tolist() +
                    rng.integers(4097, RING_CHUNKS * 4096 - 4, size=300).tolist(), dtype=np.uint64)
    rng.shuffle(lens)
    lead = 6 if mode == "log_verify" else 0
    gaps = rng.integers(0, 8, size=len(lens)).astype(np.uint64) + 4 + lead
    off = np.cumsum(np.concatenate([[5 + lead], (lens + gaps)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 16, 0x5EED00E2)
    n = len(lens)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if mode == "plain" else None
    if mode in ("verify", "log_verify"):
        raw, _ = oracle.batch(host, off, lens)
        masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
        at = (off - 6) if mode == "log_verify" else (off + lens)
        tr = at.astype(np.int64)[:, None] + np.arange(4)[None, :]
        host[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
        for v in rng.choice(n, size=8, replace=False):  # damaged spans
            host[int(off[v]) + int(lens[v]) // 2] ^= 0x40 if lens[v] else 0
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev) if init is not None else None
    crc32c.batch(buf, d_off[:1], d_len[:1])
    before = _stats(native)
    if mode == "plain":
        want, _ = oracle.batch(host, off, lens, init, mask=True)
        out, _ = crc32c.batch(buf, d_off, d_len, d_init, mask=True)
        np.testing.assert_array_equal(_u32(out), want)
    elif mode == "seal":
        raw, _ = oracle.batch(host, off, lens)
        masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
        out, _ = crc32c.batch(buf, d_off, d_len, mask=True, trailer=True)
        np.testing.assert_array_equal(_u32(out), masked)
        got = buf.cpu().numpy()
        tr = (off + lens).astype(np.int64)[:, None] + np.arange(4)[None, :]
        np.testing.assert_array_equal(got[tr].reshape(-1).view("<u4"), masked)
    else:
        log = mode == "log_verify"
        want, _ = oracle.batch(host, off, lens)
        at = (off - 6) if log else (off + lens)
        stored = host[at.astype(np.int64)[:, None] + np.arange(4)[None, :]].reshape(-1).view("<u4")
        wmm = np.array([oracle.unmask(int(x)) != int(c) for x, c in zip(stored, want)], dtype=np.uint8)
        out, mm = crc32c.batch(buf, d_off, d_len, verify=True, log_header=log)
        np.testing.assert_array_equal(_u32(out), want)
        np.testing.assert_array_equal(mm.cpu().numpy(), wmm)
        assert 0 < int(wmm.sum()) <= 8
    assert _last_split_rc(native) == -2  # the one-launch path
    assert (_stats(native) - before).tolist() == [0, 0, 0, 0]  # no tickets, no whole spans


def test_ring_batch_of_16_64k_spans(dev, oracle, native):
    """A one-launch batch of 16 KiB and 64 KiB spans (LevelDB block_size
    16/64 KiB; config 3's long sizes): all folded in the ring, no tickets
    (as one-chunk tickets such batches took tens of ms).  4096 spans, all
    checked."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00E3)
    lens = rng.choice([16384, 65536, 16384 - 5, 65536 - 9], size=4096).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens + 5)[:-1]]).astype(np.uint64) + 3
    host = oracle.synth(int(off[-1] + lens[-1]) + 16, 0x5EED00E4)
    want, _ = oracle.batch(host, off, lens)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    crc32c.batch(buf, d_off[:1], d_len[:1])
    before = _stats(native)
    out, _ = crc32c.batch(buf, d_off, d_len)
    np.testing.assert_array_equal(_u32(out), want)
    assert _last_split_rc(native) == -2
    assert (_stats(native) - before).tolist() == [0, 0, 0, 0]


def test_huge_spans_all_waves_claim(dev, oracle, native):
    """A one-launch batch of a few 24-40 MiB spans at odd offsets among short
    ones (a push of >= 1 MiB of ticket work calls every wave to claim): every
    result against the oracle, every ticket accounted for once; verify mode
    with one damaged huge span."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00E5)
    lens = np.concatenate([rng.integers(0, 4097, size=2000),
                           rng.integers(24 << 20, 40 << 20, size=5)]).astype(np.uint64)
    rng.shuffle(lens)
    off = np.cumsum(np.concatenate([[7], (lens + 4 + 3)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 16, 0x5EED00E6)
    raw, _ = oracle.batch(host, off, lens)
    masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    tr = (off + lens).astype(np.int64)[:, None] + np.arange(4)[None, :]
    host[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
    big = int(np.argmax(lens))
    host[int(off[big]) + int(lens[big]) // 2] ^= 0x02
    want, wmm = oracle.batch(host, off, lens, verify=True)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    crc32c.batch(buf, d_off[:1], d_len[:1])
    before = _stats(native)
    out, mm = crc32c.batch(buf, d_off, d_len, verify=True)
    after = _stats(native)
    assert _last_split_rc(native) == -2
    np.testing.assert_array_equal(_u32(out), want)
    np.testing.assert_array_equal(mm.cpu().numpy(), wmm)
    assert np.flatnonzero(wmm).tolist() == [big]
    expect = 0
    for L, o in zip(lens.tolist(), off.tolist()):
        h = min((4 - o % 4) % 4, L)  # the device copy starts 256-B aligned
        nch = ((L - h) // 4 + 1023) // 1024
        if nch > RING_CHUNKS:
            lg = ticket_lg(nch, len(lens))
            expect += (nch + (1 << lg) - 1) >> lg
    d = after - before
    assert d[1] == 0 and d[0] + d[2] + d[3] == expect, (d, expect)


@pytest.mark.parametrize("nspans", [1, 3])
def test_few_huge_spans_many_tickets(dev, oracle, native, nspans):
    """Batches of one 320 MiB span and of three ~100 MiB spans: fewer spans
    than waves, so a span gets up to 2 nwaves / n tickets (<= 4096; several
    Horner steps in the combine), claimed by every wave.  Results against
    the oracle, every ticket accounted for once."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00E7 + nspans)
    if nspans == 1:
        lens = np.array([(320 << 20) + 13], dtype=np.uint64)
    else:
        lens = rng.integers(90 << 20, 110 << 20, size=nspans).astype(np.uint64)
    off = np.cumsum(np.concatenate([[5], (lens + 3)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 16, 0x5EED00E8)
    init = rng.integers(0, 2**32, size=nspans, dtype=np.uint64).astype(np.uint32)
    want, _ = oracle.batch(host, off, lens, init, mask=True)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev)
    crc32c.batch(buf, d_off[:1], d_len[:1])
    before = _stats(native)
    out, _ = crc32c.batch(buf, d_off, d_len, d_init, mask=True)
    after = _stats(native)
    assert _last_split_rc(native) == -2
    np.testing.assert_array_equal(_u32(out), want)
    expect = 0
    for L, o in zip(lens.tolist(), off.tolist()):
        h = min((4 - o % 4) % 4, L)
        nch = ((L - h) // 4 + 1023) // 1024
        lg = ticket_lg(nch, nspans)
        expect += (nch + (1 << lg) - 1) >> lg
    d = after - before
    assert d[1] == 0 and d[0] + d[2] + d[3] == expect, (d, expect)
    assert expect > 64 * nspans  # more than one Horner step per span


def test_ticket_workspace_full_whole_spans(dev, oracle, native):
    """A ticket workspace of 16 entries: the first pushes fit, the rest spill
    to whole-span folding by their discovering wave; claims of null tickets
    are skipped.  Results still bit-exact."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00D5)
    lens = rng.integers(4100, 400_000, size=300).astype(np.uint64)
    lens[::3] = rng.integers(0, 4000, size=len(lens[::3]))
    off = np.cumsum(np.concatenate([[3], (lens + 5)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 16, 0x5EED00D6)
    want, _ = oracle.batch(host, off, lens)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    crc32c.batch(buf, d_off[:1], d_len[:1])
    before = _stats(native)
    prev = native.prismdb_crc32c_direct_tickets(16)
    try:
        out, _ = crc32c.batch(buf, d_off, d_len)
        got = _u32(out)
        after = _stats(native)
    finally:
        native.prismdb_crc32c_direct_tickets(prev)
    np.testing.assert_array_equal(got, want)
    assert (after - before)[1] > 0  # spans folded whole
    out2, _ = crc32c.batch(buf, d_off, d_len)  # full workspace again
    np.testing.assert_array_equal(_u32(out2), want)


@pytest.mark.parametrize("dbg", [1, 3])
def test_late_push_and_orphans(dev, oracle, native, dbg):
    """Pushes delayed ~100 us (test hook bit 0): the ticket workers have
    stopped waiting, so the late pusher claims its own tickets after its run
    (stats[3]).  With bit 1 every worker first makes one blind claim: those
    past the supply are orphans, which the pusher finds claimed and folds
    itself (stats[0]).  An SST file with sealed trailers, verify; every
    ticket accounted for exactly once."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00D7)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    crc32c.batch(buf, d_off[:1], d_len[:1])
    before = _stats(native)
    prev = native.prismdb_crc32c_direct_debug(dbg)
    try:
        out, mm = crc32c.batch(buf, d_off, d_len, verify=True, check_bounds=False)
        got, gmm = _u32(out), mm.cpu().numpy()
        after = _stats(native)
    finally:
        native.prismdb_crc32c_direct_debug(prev)
    np.testing.assert_array_equal(got, raw)
    assert (gmm == 0).all()
    d = after - before
    nch = (int(lens[-1]) + 4095) // 4096  # the index block (8-B aligned, offset multiple of 4)
    lg = ticket_lg(nch, len(lens))
    T = (nch + (1 << lg) - 1) >> lg
    assert d[0] + d[2] + d[3] == T, (d, T)
    assert d[1] == 0
    if dbg == 3:
        assert d[0] > 0  # orphans adopted
    else:
        assert d[3] > 0  # the pusher's own late claims


def test_direct_limit(dev, oracle, native):
    """2^17 spans (the one-launch limit) take one launch, 2^17 + 1 two
    windows of the same kernel, and with the windows off the planner; all
    bit-exact on the same mix of short and long spans."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00D8)
    size = 64 << 20
    host = oracle.synth(size, 0x5EED00D8)
    for n, windows, rc in ((1 << 17, 1, -2), ((1 << 17) + 1, 1, -2), ((1 << 17) + 1, 0, 0)):
        lens = rng.integers(0, 4500, size=n).astype(np.uint64)
        lens[rng.integers(0, n, size=20)] = rng.integers(4500, 200_000, size=20)
        off = rng.integers(0, size - 200_001, size=n).astype(np.uint64)
        want, _ = oracle.batch(host, off, lens)
        prev = native.prismdb_crc32c_windows(windows)
        try:
            out, _ = crc32c.batch(torch.from_numpy(host).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                                  torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev))
        finally:
            native.prismdb_crc32c_windows(prev)
        assert _last_split_rc(native) == rc
        np.testing.assert_array_equal(_u32(out), want)


def test_direct_concurrent_threads(dev, oracle):
    """Four host threads on their own streams, each enqueuing 20 one-launch
    file-sized batches back to back (per-(thread, stream) ticket workspaces and
    counters), then checking all of them."""
    import threading

    import torch
    from prismdb_amd import crc32c

    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00D9)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    errors = []

    def run(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                outs = torch.empty((20, len(off)), dtype=torch.int32, device=dev)
                for i in range(20):
                    crc32c.batch(buf, d_off, d_len, mask=bool(t & 1), out=outs[i], check_bounds=False, stream=s)
                s.synchronize()
                want = masked if t & 1 else raw
                if not (outs.cpu().numpy().view(np.uint32) == want[None, :]).all():
                    errors.append(t)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    assert not errors, errors


def test_thread_churn_device_memory_flat(dev, oracle, native):
    """64 short-lived caller threads (8 at a time), each with its own stream
    and one file-sized call -- the first half on the one-launch path, the
    second on the planner path (the route hook is set between waves, never
    by the threads) -- each thread's workspaces (> 25 MiB of device memory)
    go back when it exits (stream-ordered frees behind its last batch, pool
    trimmed), so free device memory afterwards is where it was, and the
    results are right throughout."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00DA)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    errors = []

    def run(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                out = torch.empty(len(off), dtype=torch.int32, device=dev)
                crc32c.batch(buf, d_off, d_len, out=out, check_bounds=False, stream=s)
                s.synchronize()
                if not (out.cpu().numpy().view(np.uint32) == raw).all():
                    errors.append(t)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    def wave(first):
        th = [threading.Thread(target=run, args=(first + t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)

    prev = native.prismdb_crc32c_direct_max(1 << 17)
    try:
        wave(0)  # torch's own per-thread state and the tensors above exist from here on
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        free0, _ = torch.cuda.mem_get_info(dev)
        for w in range(1, 8):
            if w == 4:
                native.prismdb_crc32c_direct_max(0)  # the planner path from here on
            wave(8 * w)
    finally:
        native.prismdb_crc32c_direct_max(prev)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free1, _ = torch.cuda.mem_get_info(dev)
    assert not errors, errors
    # 56 leaked thread workspaces would be > 1.4 GiB
    assert free0 - free1 < 256 << 20, (free0 - free1) / 2**20


def test_unordered_first_call_and_tag_wrap(dev, oracle, native):
    """PRISMDB_CRC32C_UNORDERED (accepted, no effect) as the FIRST call on a
    fresh stream -- right behind the ticket workspace's zero-fill -- on SST
    files whose index span is cut into tickets; then the workspace's call
    count is set just below the 16-bit tag wrap (test hook), and five more
    ticketed calls cross it (the wrap zeroes the workspace again between
    two calls).  Every result, verify flag and trailer against the oracle."""
    import torch
    from prismdb_amd import crc32c

    nf = 2
    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00DC, files=nf)
    per = len(off) // nf
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        buf = torch.from_numpy(host).to(dev)
        d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        outs = torch.full((7, per), 7, dtype=torch.int32, device=dev)
        mms = torch.full((7, per), 7, dtype=torch.uint8, device=dev)

    def call(i, f, verify):
        sl = slice(f * per, (f + 1) * per)
        if verify:
            crc32c.batch(buf, d_off[sl], d_len[sl], verify=True, out=outs[i], mismatch=mms[i], check_bounds=False,
                         unordered=True, stream=s)
        else:
            crc32c.batch(buf, d_off[sl], d_len[sl], mask=True, trailer=True, out=outs[i], check_bounds=False,
                         unordered=True, stream=s)

    call(0, 0, False)  # the stream's first call: workspace allocated and zeroed, then this launch
    s.synchronize()
    sp = ctypes.c_void_p(int(s.cuda_stream))
    assert native.prismdb_crc32c_direct_set_gen(sp, 0xFFFD) == 0
    plan = [(1, 1, True), (2, 0, False), (3, 1, False), (4, 0, True), (5, 1, True), (6, 0, True)]
    for i, f, v in plan:  # tags 0xFFFE, 0xFFFF, wrap (zero-fill) -> 1, 2, 3, 4
        call(i, f, v)
    s.synchronize()
    assert _last_split_rc(native) == -2
    got = outs.cpu().numpy().view(np.uint32)
    mm = mms.cpu().numpy()
    for i, f, v in [(0, 0, False)] + plan:
        want = (raw if v else masked)[f * per:(f + 1) * per]
        np.testing.assert_array_equal(got[i], want, err_msg=f"call {i}")
        if v:
            assert not mm[i].any(), f"call {i}"
    assert (buf.cpu().numpy() == host).all()


def test_unordered_file_calls(dev, oracle, native):
    """PRISMDB_CRC32C_UNORDERED (accepted and ignored: every launch is in
    stream order): 24 SST files sealed one call each, back to back, then all
    verified the same way, then a verify right after a flagged reseal of the
    same file.  Every result, every trailer and every verify flag against the
    oracle."""
    import torch
    from prismdb_amd import crc32c

    nf = 24
    host, off, lens, raw, masked = _sst_file(oracle, 0x5EED00DB, files=nf)
    sealed = host.copy()
    tr = (off + lens.astype(np.uint64)).astype(np.int64)[:, None] + np.arange(4)[None, :]
    host[tr] = 0  # trailers to be written
    buf = torch.from_numpy(host).to(dev)
    per = len(off) // nf
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    outs = torch.empty((3, len(off)), dtype=torch.int32, device=dev)
    mms = torch.full((2, len(off)), 7, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for f in range(nf):
        sl = slice(f * per, (f + 1) * per)
        crc32c.batch(buf, d_off[sl], d_len[sl], mask=True, trailer=True, out=outs[0, sl], check_bounds=False,
                     unordered=True)
    for f in range(nf):
        sl = slice(f * per, (f + 1) * per)
        crc32c.batch(buf, d_off[sl], d_len[sl], verify=True, out=outs[1, sl], mismatch=mms[0, sl],
                     check_bounds=False, unordered=True)
    # ordered after unordered: file 0 resealed unordered, then verified in order
    crc32c.batch(buf, d_off[:per], d_len[:per], mask=True, trailer=True, out=outs[2, :per], check_bounds=False,
                 unordered=True)
    crc32c.batch(buf, d_off[:per], d_len[:per], verify=True, out=outs[2, per:2 * per], mismatch=mms[1, :per],
                 check_bounds=False)
    torch.cuda.synchronize()
    assert _last_split_rc(native) == -2  # the one-launch path
    got = outs.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got[0], masked)
    np.testing.assert_array_equal(got[1], raw)
    np.testing.assert_array_equal(got[2, :per], masked[:per])
    np.testing.assert_array_equal(got[2, per:2 * per], raw[:per])
    assert not mms.cpu().numpy()[0].any() and not mms.cpu().numpy()[1, :per].any()
    assert (buf.cpu().numpy() == sealed).all()  # every trailer as the reference writes it


@pytest.mark.parametrize("seed", range(8))
def test_direct_random_batches(dev, oracle, native, seed):
    """Random one-launch batches: 1 to 20 000 spans mixing every length class
    the kernel treats differently -- empty and short spans, ring spans of 2
    to 32 chunks, ticket spans (33 chunks to a few MiB), now and then one or
    two of tens of MiB (help flag, idle groups claiming, batch-scaled
    tickets) -- at any alignment, in a random mode: plain with init, MASK,
    verify (a few damaged), or sealing.  Every result against the oracle,
    every ticket accounted for exactly once."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED0F00 + seed)
    n = int(rng.choice([1, 2, 5, 40, 300, 3000, 20000]))
    p = [0.55, 0.2, 0.15, 0.09, 0.01] if n < 3000 else [0.8, 0.16, 0.035, 0.005, 0.0]
    cls = rng.choice(5, size=n, p=p)
    lens = np.where(cls == 0, rng.integers(0, 4097, size=n),
           np.where(cls == 1, rng.integers(4097, RING_CHUNKS * 4096 - 4, size=n),
           np.where(cls == 2, rng.integers(RING_CHUNKS * 4096, 1 << 20, size=n),
           np.where(cls == 3, rng.integers(1 << 20, 4 << 20, size=n),
                    rng.integers(16 << 20, 40 << 20, size=n))))).astype(np.uint64)
    while int(lens.sum()) > (400 << 20):  # keep the case small: shrink the largest span
        lens[int(np.argmax(lens))] //= 4
    mode = ["plain", "mask", "verify", "seal"][int(rng.integers(0, 4))]
    gaps = rng.integers(4, 12, size=n).astype(np.uint64)
    off = np.cumsum(np.concatenate([[int(rng.integers(0, 8))], (lens + gaps)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1] + lens[-1]) + 16, 0x5EED0F80 + seed)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if mode == "plain" else None
    raw, _ = oracle.batch(host, off, lens)
    masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    if mode == "verify":
        tr = (off + lens).astype(np.int64)[:, None] + np.arange(4)[None, :]
        host[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
        for v in rng.choice(n, size=min(n, 3), replace=False):
            if lens[v]:
                host[int(off[v]) + int(rng.integers(0, int(lens[v])))] ^= 0x10
        raw, _ = oracle.batch(host, off, lens)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev) if init is not None else None
    crc32c.batch(buf, d_off[:1], d_len[:1])
    before = _stats(native)
    if mode == "plain":
        want, _ = oracle.batch(host, off, lens, init)
        out, _ = crc32c.batch(buf, d_off, d_len, d_init)
        np.testing.assert_array_equal(_u32(out), want)
    elif mode == "mask":
        out, _ = crc32c.batch(buf, d_off, d_len, mask=True)
        np.testing.assert_array_equal(_u32(out), masked)
    elif mode == "verify":
        want, wmm = oracle.batch(host, off, lens, verify=True)
        out, mm = crc32c.batch(buf, d_off, d_len, verify=True)
        np.testing.assert_array_equal(_u32(out), want)
        np.testing.assert_array_equal(mm.cpu().numpy(), wmm)
    else:
        out, _ = crc32c.batch(buf, d_off, d_len, mask=True, trailer=True)
        np.testing.assert_array_equal(_u32(out), masked)
        got = buf.cpu().numpy()
        tr = (off + lens).astype(np.int64)[:, None] + np.arange(4)[None, :]
        np.testing.assert_array_equal(got[tr].reshape(-1).view("<u4"), masked)
    after = _stats(native)
    assert _last_split_rc(native) == -2
    expect = 0
    for L, o in zip(lens.tolist(), off.tolist()):
        h = min((4 - o % 4) % 4, L)  # the device copy starts 256-B aligned
        nch = ((L - h) // 4 + 1023) // 1024
        if nch > RING_CHUNKS:
            lg = ticket_lg(nch, n)
            expect += (nch + (1 << lg) - 1) >> lg
    d = after - before
    assert d[1] == 0 and d[0] + d[2] + d[3] == expect, (d, expect, n, mode)


@pytest.mark.parametrize("mode", ["plain", "seal", "verify"])
def test_bulk_windows(dev, oracle, native, mode):
    """A batch of 300 000 spans (> 2^17) as windows of the one-launch kernel
    (the windows hook on), back to back on a caller stream that first
    uploads the bytes: the windows start after the upload, the results are
    read on that stream right after the call, and every result,
    trailer and verify flag equals the oracle's.  Lengths 0-8000 B at any
    alignment with random init, and 40 spans of 0.2-2 MiB (tickets)."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0x5EED00E0 + len(mode))
    n = 300_000
    lens = rng.integers(0, 8000, size=n).astype(np.uint32)
    lens[rng.choice(n, size=40, replace=False)] = rng.integers(200_000, 2_000_000, size=40)
    gaps = rng.integers(4, 12, size=n).astype(np.uint64)  # room for a trailer after each span
    off = (np.cumsum(lens.astype(np.uint64) + gaps) - lens.astype(np.uint64) - gaps + 16).astype(np.uint64)
    host = oracle.synth(int(off[-1]) + int(lens[-1]) + 64, 0x5EED00E1)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if mode == "plain" else None
    raw, _ = oracle.batch(host, off, lens, init)
    masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    tr = (off + lens.astype(np.uint64)).astype(np.int64)[:, None] + np.arange(4)[None, :]
    if mode == "verify":
        host[tr] = masked.astype("<u4").view(np.uint8).reshape(-1, 4)
        bad = rng.choice(n, size=5, replace=False)
        for i in bad:
            host[int(off[i])] ^= 0x11  # (an empty span: its stored crc's first byte)
        raw, _ = oracle.batch(host, off, lens)
        masked = np.array([oracle.mask(int(c)) for c in raw], dtype=np.uint32)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        buf = torch.empty(len(host), dtype=torch.uint8, device=dev)
        buf.copy_(torch.from_numpy(host).pin_memory(), non_blocking=True)
        d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        d_init = torch.from_numpy(init.view(np.int32)).to(dev) if init is not None else None
        out = torch.full((n,), 7, dtype=torch.int32, device=dev)
        mm = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    prev = native.prismdb_crc32c_windows(1)
    try:
        if mode == "plain":
            crc32c.batch(buf, d_off, d_len, d_init, out=out, stream=s, check_bounds=False)
        elif mode == "seal":
            crc32c.batch(buf, d_off, d_len, mask=True, trailer=True, out=out, stream=s, check_bounds=False)
        else:
            crc32c.batch(buf, d_off, d_len, verify=True, out=out, mismatch=mm, stream=s, check_bounds=False)
    finally:
        native.prismdb_crc32c_windows(prev)
    with torch.cuda.stream(s):
        got, gmm, gbuf = out.clone(), mm.clone(), buf[:16].clone() if mode != "seal" else buf.clone()
    s.synchronize()
    assert _last_split_rc(native) == -2  # one-launch windows
    np.testing.assert_array_equal(_u32(got), masked if mode == "seal" else raw)
    if mode == "seal":
        sealed = gbuf.cpu().numpy()
        np.testing.assert_array_equal(sealed[tr].copy().view("<u4").reshape(-1), masked)
    if mode == "verify":
        want_bad = np.zeros(n, dtype=np.uint8)
        want_bad[bad] = 1
        np.testing.assert_array_equal(gmm.cpu().numpy(), want_bad)
