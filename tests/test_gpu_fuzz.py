"""Randomized parity of the batch engine against the oracle: random span
geometries (empty to split-path lengths, any alignment, overlapping), random
flags (MASK, verify, WRITE_TRAILER, LOG_HEADER) and random fixed-stride
shapes, on the fast and on the generic kernel, and descriptor batches on
every route: the one-launch kernel, and the planner path with the lane kernel
in front of every batch, of log batches only, or of none.  Bit-exact.

Expected values come from the oracle (oracle/crc32c_oracle.c, pinned to the
reference's golden vectors) on the same bytes; what a flag adds is checked
by its definition at the call sites:
  verify       Unmask(LE32(span end)) == crc          table/format.cc:93-101
  LOG_HEADER   the stored crc sits 6 bytes before the span  db/log_reader.cc:246-257
  WRITE_TRAILER  LE32(Mask(crc)) written at the span end  table/table_builder.cc:194-196
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# PRISMDB_FUZZ_SEEDS widens a campaign (the default keeps the suite short)
SEEDS = list(range(int(os.environ.get("PRISMDB_FUZZ_SEEDS", "24"))))


@pytest.fixture(scope="module")
def dev(native):
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    from prismdb_amd import crc32c

    crc32c.device_init(0)
    return torch.device("cuda", 0)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _lengths(rng, n):
    kind = rng.integers(0, 6, size=n)
    lens = np.select(
        [kind == 0, kind == 1, kind == 2, kind == 3, kind == 4],
        [rng.integers(0, 9, size=n), rng.integers(9, 400, size=n), rng.integers(4088, 4105, size=n),
         rng.integers(1, 17, size=n) * 4096, rng.integers(400, 70_000, size=n)],
        rng.integers(130_000, 300_000, size=n))
    # split-path spans (> 128 KiB) are a minority
    big = lens > 131072
    keep = rng.random(n) < 0.1
    lens[big & ~keep] = lens[big & ~keep] % 9000
    return lens.astype(np.uint64)


@pytest.mark.parametrize("seed", SEEDS)
def test_random_spans(dev, oracle, any_route, seed):
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0xF0220000 + seed)
    n = int(rng.choice([1, 2, 63, 64, 65, 500, 3000, 20000]))
    size = 8 << 20
    host = oracle.synth(size, 0xF0220000 + seed)
    lens = _lengths(rng, n)
    off = rng.integers(8, size - int(lens.max()) - 8, size=n).astype(np.uint64)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.5 else None
    mask = bool(rng.random() < 0.5)
    verify = bool(rng.random() < 0.5)
    log_header = verify and bool(rng.random() < 0.5)
    if verify:
        # plant correct stored crcs for a third of the spans (stores may land in other spans)
        want, _ = oracle.batch(host, off, lens, init)
        for i in np.nonzero(rng.random(n) < 0.33)[0]:
            o = int(off[i]) - 6 if log_header else int(off[i] + lens[i])
            host[o:o + 4] = np.frombuffer(np.uint32(oracle.mask(int(want[i]))).tobytes(), dtype=np.uint8)
    want, _ = oracle.batch(host, off, lens, init, mask=mask)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev) if init is not None else None
    out, mm = crc32c.batch(buf, d_off, d_len, d_init, mask=mask, verify=verify, log_header=log_header)
    np.testing.assert_array_equal(_u32(out), want)
    if verify:
        raw, _ = oracle.batch(host, off, lens, init)
        pos = off.astype(np.int64) - 6 if log_header else (off + lens).astype(np.int64)
        stored = host[pos[:, None] + np.arange(4)[None, :]].copy().view("<u4").reshape(-1)
        bad = np.array([oracle.unmask(int(s)) != int(r) for s, r in zip(stored, raw)], dtype=np.uint8)
        np.testing.assert_array_equal(mm.cpu().numpy(), bad)


@pytest.mark.parametrize("seed", SEEDS[:12])
def test_random_trailer_sealing(dev, oracle, any_route, seed):
    """WRITE_TRAILER on disjoint spans (a trailer must not land in another
    span): every trailer is LE32(Mask(crc)) or the raw crc, per MASK; bytes
    outside the trailers are untouched; LOG_HEADER writes 6 bytes before."""
    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0xF0230000 + seed)
    n = int(rng.choice([1, 5, 64, 700, 5000]))
    lens = _lengths(rng, n)
    log_header = bool(rng.random() < 0.5)
    mask = bool(rng.random() < 0.7)
    gaps = rng.integers(10, 40, size=n).astype(np.uint64)  # room for the 4-byte field on either side
    off = np.cumsum(np.concatenate([[16], (lens + gaps)[:-1]])).astype(np.uint64)
    size = int(off[-1] + lens[-1]) + 64
    host = oracle.synth(size, 0xF0230000 + seed)
    want, _ = oracle.batch(host, off, lens, None, mask=mask)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    out, _ = crc32c.batch(buf, d_off, d_len, mask=mask, trailer=True, log_header=log_header)
    np.testing.assert_array_equal(_u32(out), want)
    got = buf.cpu().numpy()
    pos = off.astype(np.int64) - 6 if log_header else (off + lens).astype(np.int64)
    idx = (pos[:, None] + np.arange(4)[None, :]).reshape(-1)
    np.testing.assert_array_equal(got[idx].view("<u4"), want)
    keep = np.ones(size, dtype=bool)
    keep[idx] = False
    np.testing.assert_array_equal(got[keep], host[keep])


@pytest.mark.parametrize("seed", SEEDS)
def test_random_fixed_geometry(dev, oracle, native, seed):
    """Random fixed-stride batches through both kernels (forced generic too)."""
    import ctypes

    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0xF0240000 + seed)
    length = int(rng.choice([0, 1, 3, 4, 8, 252, 256, 260, 1024, 2044, 3988, 4092, 4096, 5000, 70_000]))
    stride = length + int(rng.choice([0, 1, 4, 5, 8, 100]))
    stride = max(stride, 1)
    nblk = int(rng.integers(1, max(2, min(20_000, (16 << 20) // stride))))
    base = int(rng.choice([0, 4, 1, 2]))
    total = base + (nblk - 1) * stride + length + 8
    host = oracle.synth(total, 0xF0240000 + seed)
    init = int(rng.integers(0, 2**32))
    mask = bool(rng.random() < 0.5)
    want = oracle.batch_fixed(host[base:], stride, length, nblk, init=init, mask=mask)
    buf = torch.from_numpy(host).to(dev)
    for force in (0, 1):
        native.prismdb_crc32c_force_generic.argtypes = [ctypes.c_int]
        native.prismdb_crc32c_force_generic(force)
        try:
            out, _ = crc32c.batch_fixed(buf[base:], stride, length, nblk, init=init, mask=mask)
            np.testing.assert_array_equal(_u32(out), want)
        finally:
            native.prismdb_crc32c_force_generic(0)


@pytest.mark.parametrize("seed", SEEDS[:max(4, len(SEEDS) // 3)])
def test_random_pair_batches(dev, oracle, native, seed, planner_bulk):
    """Random batches the pair-run span kernel takes: >= 2^18 spans, each one
    task (0..4096 B at any alignment) or long (split path, 1 in 2000), at
    random overlapping offsets; random init, MASK, and VERIFY against stored
    crcs planted for a third of the spans.  The split counters confirm the
    batch went to the span pass with no overflow."""
    import ctypes

    import torch
    from prismdb_amd import crc32c

    rng = np.random.default_rng(0xF0250000 + seed)
    n = int(rng.choice([1 << 18, (1 << 18) + 1, (1 << 18) + 63, 300_001]))
    size = 32 << 20
    host = oracle.synth(size, 0xF0250000 + seed)
    kind = rng.integers(0, 4, size=n)
    lens = np.select([kind == 0, kind == 1, kind == 2], [rng.integers(0, 9, size=n), rng.integers(9, 1300, size=n),
                                                         rng.integers(3800, 4097, size=n)], rng.integers(1300, 3800, size=n))
    lens[rng.random(n) < 0.0005] = rng.integers(131073, 600_000)
    lens = lens.astype(np.uint64)
    off = rng.integers(8, size - int(lens.max()) - 8, size=n).astype(np.uint64)
    init = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.5 else None
    mask = bool(rng.random() < 0.5)
    verify = bool(rng.random() < 0.5)
    if verify:
        want, _ = oracle.batch(host, off, lens, init)
        for i in np.nonzero(rng.random(n) < 0.33)[0]:
            o = int(off[i] + lens[i])
            host[o:o + 4] = np.frombuffer(np.uint32(oracle.mask(int(want[i]))).tobytes(), dtype=np.uint8)
    want, _ = oracle.batch(host, off, lens, init, mask=mask)
    buf = torch.from_numpy(host).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev)
    d_init = torch.from_numpy(init.view(np.int32)).to(dev) if init is not None else None
    out, mm = crc32c.batch(buf, d_off, d_len, d_init, mask=mask, verify=verify)
    arr = (ctypes.c_uint64 * 4)()
    native.prismdb_crc32c_last_split.argtypes = [ctypes.c_void_p]
    assert native.prismdb_crc32c_last_split(arr) == 0 and arr[2] == 0
    sched = (ctypes.c_uint64 * 3)()
    native.prismdb_crc32c_last_schedule.argtypes = [ctypes.c_void_p]
    assert native.prismdb_crc32c_last_schedule(sched) == 0
    assert sched[1] == 0 and sched[2] == 1, list(sched)  # the pair-run kernel took the batch
    np.testing.assert_array_equal(_u32(out), want)
    if verify:
        raw, _ = oracle.batch(host, off, lens, init)
        pos = (off + lens).astype(np.int64)
        stored = host[pos[:, None] + np.arange(4)[None, :]].copy().view("<u4").reshape(-1)
        bad = np.array([oracle.unmask(int(x)) != int(r) for x, r in zip(stored, raw)], dtype=np.uint8)
        np.testing.assert_array_equal(mm.cpu().numpy(), bad)
