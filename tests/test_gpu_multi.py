"""leveldb_crc32c_batch_multi: partitions on several devices of one process,
results gathered over RCCL to the first device (include/prismdb_crc32c.h;
PrismDB's per-partition background threads, db/db_impl.h:359).  On the
1-GPU lease this runs at ndev = 1 (the clique, its streams, the scratch and
the caller-stream handoff, with the gather a no-op); with more visible
devices also across all of them.  Bit-exact against the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _partition(oracle, seed, nblocks, long_every=0):
    """An SST-shaped partition: 3988-B data spans at stride 3992 with every
    `long_every`-th span a long (index-like) one, each followed by its
    4-byte trailer."""
    rng = np.random.default_rng(seed)
    lens = np.full(nblocks, 3988, dtype=np.uint32)
    if long_every:
        lens[::long_every] = rng.integers(5000, 300_000, size=len(lens[::long_every]))
    off = np.cumsum(np.concatenate([[8], (lens.astype(np.uint64) + 4)[:-1]])).astype(np.uint64)
    host = oracle.synth(int(off[-1]) + int(lens[-1]) + 64, seed)
    return host, off, lens


def _to(dev, host, off, lens):
    import torch

    return (torch.from_numpy(host).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
            torch.from_numpy(lens.view(np.int32)).to(dev))


@pytest.fixture(scope="module")
def devices(native):
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return list(range(torch.cuda.device_count()))


@pytest.mark.parametrize("long_every", [0, 97])
def test_multi_one_device_seal_then_verify(devices, oracle, long_every):
    """ndev = 1: seal (MASK | WRITE_TRAILER) one partition, then verify it;
    then damage three blocks and verify again."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens = _partition(oracle, 0x5EED0301 + long_every, 5000, long_every)
    want, _ = oracle.batch(host, off, lens, mask=True)
    dev = torch.device("cuda", devices[0])
    buf, d_off, d_len = _to(dev, host, off, lens)
    out, _ = crc32c.batch_multi([(buf, d_off, d_len)], mask=True, trailer=True)
    np.testing.assert_array_equal(_u32(out), want)
    sealed = buf.cpu().numpy()
    tr = (off + lens.astype(np.uint64)).astype(np.int64)
    np.testing.assert_array_equal(
        sealed[tr[:, None] + np.arange(4)[None, :]].copy().view("<u4").reshape(-1), want)
    raw, _ = oracle.batch(host, off, lens)
    out, mm = crc32c.batch_multi([(buf, d_off, d_len)], verify=True)
    np.testing.assert_array_equal(_u32(out), raw)
    assert not mm.cpu().numpy().any()
    bad = [0, 1234, 4999]
    for i in bad:
        buf[int(off[i]) + 7] ^= 0x40
    out, mm = crc32c.batch_multi([(buf, d_off, d_len)], verify=True)
    assert sorted(np.nonzero(mm.cpu().numpy())[0].tolist()) == bad


def test_multi_one_device_streams_and_init(devices, oracle):
    """ndev = 1 on a side stream with per-span initial registers: the call
    orders after work already on the stream (the buffer is filled there) and
    the stream waits for the results; repeated calls grow nothing."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens = _partition(oracle, 0x5EED0303, 3000, 50)
    init = np.random.default_rng(3).integers(0, 2**32, size=len(off), dtype=np.uint64).astype(np.uint32)
    want, _ = oracle.batch(host, off, lens, init, mask=True)
    dev = torch.device("cuda", devices[0])
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        buf = torch.empty(len(host), dtype=torch.uint8, device=dev)
        buf.copy_(torch.from_numpy(host).pin_memory(), non_blocking=True)
        d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        d_init = torch.from_numpy(init.view(np.int32)).to(dev)
    for _ in range(3):
        out, _ = crc32c.batch_multi([(buf, d_off, d_len, d_init)], mask=True, streams=[s], check_bounds=False)
        with torch.cuda.stream(s):
            got = out.clone()
        s.synchronize()
        np.testing.assert_array_equal(_u32(got), want)


def test_multi_all_devices(devices, oracle):
    """Every visible device one partition (different sizes, one empty when
    there are three or more); results gathered to the first, partition after
    partition."""
    import torch
    from prismdb_amd import crc32c

    if len(devices) < 2:
        pytest.skip("one visible device: ndev = 1 is covered above")
    parts, want = [], []
    for k, d in enumerate(devices):
        nb = 0 if (k == 2) else 1000 + 777 * k
        if nb == 0:
            dev = torch.device("cuda", d)
            parts.append((torch.zeros(64, dtype=torch.uint8, device=dev), torch.zeros(0, dtype=torch.int64, device=dev),
                          torch.zeros(0, dtype=torch.int32, device=dev)))
            continue
        host, off, lens = _partition(oracle, 0x5EED0310 + k, nb, 40)
        w, _ = oracle.batch(host, off, lens, mask=True)
        want.append(w)
        parts.append(_to(torch.device("cuda", d), host, off, lens))
    out, _ = crc32c.batch_multi(parts, mask=True)
    assert out.device.index == devices[0]
    np.testing.assert_array_equal(_u32(out), np.concatenate(want))


def test_multi_failure_hands_streams_back(devices, oracle, native):
    """An injected failure right after partition 0's batch is enqueued (test
    hook prismdb_crc32c_multi_fail_after): the call raises, and the caller's
    stream still waits for the clique's work -- a fill of `out` enqueued on
    it right after the failed call lands after the batch's writes, every
    entry.  The next call succeeds with its own results."""
    import torch
    from prismdb_amd import crc32c
    from prismdb_amd._lib import NativeLibraryError

    dev = torch.device("cuda", devices[0])
    nb = 1 << 18  # 1 GiB of 4 KiB spans: still running when the call returns
    host = oracle.synth(nb * 4096 + 64, 0x5EED0320)
    off = np.arange(nb, dtype=np.uint64) * 4096
    lens = np.full(nb, 4096, dtype=np.uint32)
    buf, d_off, d_len = _to(dev, host, off, lens)
    out = torch.zeros(nb, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    prev = native.prismdb_crc32c_multi_fail_after(0)
    try:
        with pytest.raises(NativeLibraryError, match="injected failure"):
            crc32c.batch_multi([(buf, d_off, d_len)], out=out, check_bounds=False)
        out.fill_(0x5A5A5A5A)  # on the caller's stream: after the failed call's batch
    finally:
        native.prismdb_crc32c_multi_fail_after(prev)
    torch.cuda.synchronize()
    assert bool((out == 0x5A5A5A5A).all())
    want, _ = oracle.batch(host[:64 * 4096], off[:64], lens[:64])
    out2, _ = crc32c.batch_multi([(buf, d_off, d_len)], check_bounds=False)
    got = _u32(out2)
    np.testing.assert_array_equal(got[:64], want)
    assert len(np.unique(got)) > nb - 64  # every span its own result, not a leftover fill


def test_multi_failure_after_second_partition(devices, oracle, native):
    """With two or more devices: an injected failure right after partition
    1's batch is enqueued (fail_after = 1) makes every enqueued partition's
    caller stream wait for the clique's work -- a fill enqueued on each right
    after the failed call lands after that partition's batch -- and the next
    call gathers every partition's own results.  (Unverified on a 1-GPU
    lease: skipped there; the driver's multi-GPU node runs it.)"""
    import torch
    from prismdb_amd import crc32c
    from prismdb_amd._lib import NativeLibraryError

    if len(devices) < 2:
        pytest.skip("needs two devices")
    nb = 1 << 17
    parts, bufs, want = [], [], []
    for k, d in enumerate(devices[:2]):
        dev = torch.device("cuda", d)
        host = oracle.synth(nb * 4096 + 64, 0x5EED0330 + k)
        off = np.arange(nb, dtype=np.uint64) * 4096
        lens = np.full(nb, 4096, dtype=np.uint32)
        parts.append(_to(dev, host, off, lens))
        want.append(oracle.batch(host[:64 * 4096], off[:64], lens[:64])[0])
        bufs.append(torch.zeros(16, dtype=torch.int32, device=dev))
    for d in devices[:2]:
        torch.cuda.synchronize(d)
    prev = native.prismdb_crc32c_multi_fail_after(1)
    try:
        with pytest.raises(NativeLibraryError, match="injected failure"):
            crc32c.batch_multi(parts, check_bounds=False)
        for b in bufs:  # on each device's current stream: after the failed call's work there
            with torch.cuda.device(b.device):
                b.fill_(7)
    finally:
        native.prismdb_crc32c_multi_fail_after(prev)
    for d in devices[:2]:
        torch.cuda.synchronize(d)
    assert all(bool((b == 7).all()) for b in bufs)
    out, _ = crc32c.batch_multi(parts, check_bounds=False)
    got = _u32(out)
    np.testing.assert_array_equal(got[:64], want[0])
    np.testing.assert_array_equal(got[nb:nb + 64], want[1])


def test_multi_timing_diagnostics(devices, oracle):
    """prismdb_crc32c_multi_timing: after a batch_multi call, one batch time
    and one gather time per device of the clique (HIP events on the clique's
    streams) and the clique's ncclCommInitAll wall time; None for a device
    list that has no clique."""
    import torch
    from prismdb_amd import crc32c

    dev = torch.device("cuda", devices[0])
    host, off, lens = _partition(oracle, 0x5EED0340, 20000, 0)
    crc32c.batch_multi([_to(dev, host, off, lens)], mask=True)
    torch.cuda.synchronize()
    tm = crc32c.multi_timing([devices[0]])
    assert tm is not None and len(tm["batch_ms"]) == 1 and len(tm["gather_ms"]) == 1
    assert tm["batch_ms"][0] > 0.0 and tm["gather_ms"][0] >= 0.0 and tm["init_ms"] > 0.0
    assert crc32c.multi_timing([devices[0], 63]) is None


@pytest.fixture
def self_gather(native):
    """prismdb_crc32c_multi_self_gather on: partition 0 is enqueued by a
    worker thread and its results reach out0 through the grouped
    ncclSend / ncclRecv to itself."""
    prev = native.prismdb_crc32c_multi_self_gather(1)
    assert native.prismdb_crc32c_multi_self_gather(1) == 1, "test hooks are off"
    yield
    native.prismdb_crc32c_multi_self_gather(prev)


@pytest.mark.parametrize("long_every", [0, 61])
def test_multi_self_gather_one_device(devices, oracle, native, self_gather, long_every):
    """The gather's RCCL call sequence on a one-device clique: partition 0's
    batch enqueued by its worker thread into clique scratch, then grouped
    ncclSend / ncclRecv of the 4-byte results and of the verify flags to
    itself (comm, stream and counts as for a partition p > 0).  Seal, verify
    and damaged verify, each bit-exact against the oracle; 20 calls back to
    back through the same worker; the host timing diagnostics after them."""
    import torch
    from prismdb_amd import crc32c

    host, off, lens = _partition(oracle, 0x5EED0350 + long_every, 30000, long_every)
    want, _ = oracle.batch(host, off, lens, mask=True)
    raw, _ = oracle.batch(host, off, lens)
    dev = torch.device("cuda", devices[0])
    buf, d_off, d_len = _to(dev, host, off, lens)
    out = torch.full((len(off) + 5,), 0x3C3C3C3C, dtype=torch.int32, device=dev)
    crc32c.batch_multi([(buf, d_off, d_len)], mask=True, trailer=True, out=out)
    got = _u32(out)
    np.testing.assert_array_equal(got[:len(off)], want)
    assert (got[len(off):] == 0x3C3C3C3C).all()  # nothing past the partition's results
    outs = [torch.empty(len(off), dtype=torch.int32, device=dev) for _ in range(20)]
    mms = [torch.full((len(off),), 9, dtype=torch.uint8, device=dev) for _ in range(20)]
    for o, m in zip(outs, mms):
        crc32c.batch_multi([(buf, d_off, d_len)], verify=True, out=o, mismatch=m, check_bounds=False)
    torch.cuda.synchronize()
    for o, m in zip(outs, mms):
        np.testing.assert_array_equal(_u32(o), raw)
        assert not m.cpu().numpy().any()
    ht = crc32c.multi_host_timing([devices[0]])
    assert ht is not None and ht["enqueue_us"][0] > 0 and ht["call_us"] >= ht["enqueue_us"][0]
    bad = [5, len(off) // 2, len(off) - 1]
    for i in bad:
        buf[int(off[i]) + 3] ^= 0x08
    out, mm = crc32c.batch_multi([(buf, d_off, d_len)], verify=True)
    assert sorted(np.flatnonzero(mm.cpu().numpy()).tolist()) == bad


def test_multi_self_gather_failure_hands_back(devices, oracle, native, self_gather):
    """Under the self-gather hook, an injected failure after partition 0's
    batch (enqueued by its worker): the call raises with the worker's
    message on the calling thread, the caller's stream still waits for the
    batch, and the next call gathers its own results."""
    import torch
    from prismdb_amd import crc32c
    from prismdb_amd._lib import NativeLibraryError

    dev = torch.device("cuda", devices[0])
    host, off, lens = _partition(oracle, 0x5EED0360, 20000, 0)
    want, _ = oracle.batch(host, off, lens)
    buf, d_off, d_len = _to(dev, host, off, lens)
    out = torch.zeros(len(off), dtype=torch.int32, device=dev)
    prev = native.prismdb_crc32c_multi_fail_after(0)
    try:
        with pytest.raises(NativeLibraryError, match="injected failure"):
            crc32c.batch_multi([(buf, d_off, d_len)], out=out, check_bounds=False)
        out.fill_(0x5A5A5A5A)
    finally:
        native.prismdb_crc32c_multi_fail_after(prev)
    torch.cuda.synchronize()
    assert bool((out == 0x5A5A5A5A).all())
    out2, _ = crc32c.batch_multi([(buf, d_off, d_len)], check_bounds=False)
    np.testing.assert_array_equal(_u32(out2), want)


def test_multi_host_enqueue_timing(devices, oracle):
    """prismdb_crc32c_multi_host_timing after a config-5-shaped planner-path
    call (> 2^18 spans): partition 0's enqueue time and start offset, and
    the whole call's host time; the enqueue is a small fraction of the
    device batch (the skew bound the workers exist for)."""
    import torch
    from prismdb_amd import crc32c

    dev = torch.device("cuda", devices[0])
    nb = 300_000
    off = np.arange(nb, dtype=np.uint64) * 3992 + 8
    lens = np.full(nb, 3988, dtype=np.uint32)
    buf = torch.empty(int(off[-1]) + 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0370)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(nb, dtype=torch.int32, device=dev)
    for _ in range(3):
        crc32c.batch_multi([(buf, d_off, d_len)], mask=True, trailer=True, out=out, check_bounds=False)
    torch.cuda.synchronize()
    ht = crc32c.multi_host_timing([devices[0]])
    tm = crc32c.multi_timing([devices[0]])
    assert ht is not None and tm is not None
    assert 0 < ht["enqueue_us"][0] < 1e3 * tm["batch_ms"][0]
    assert ht["start_us"][0] >= 0 and ht["call_us"] >= ht["enqueue_us"][0]
    print("host enqueue us", ht, "device batch ms", tm["batch_ms"])


def test_multi_rejects_bad_outputs(devices):
    """out / mismatch shorter than the partitions' total, of the wrong dtype
    or not on the root device are rejected before the C ABI writes them."""
    import torch
    from prismdb_amd import crc32c

    dev = torch.device("cuda", devices[0])
    buf = torch.zeros(4096 * 4, dtype=torch.uint8, device=dev)
    off = torch.arange(4, dtype=torch.int64, device=dev) * 4096
    lens = torch.full((4,), 4092, dtype=torch.int32, device=dev)
    for bad in (torch.zeros(3, dtype=torch.int32, device=dev), torch.zeros(4, dtype=torch.int64, device=dev),
                torch.zeros(4, dtype=torch.int32)):
        with pytest.raises(ValueError):
            crc32c.batch_multi([(buf, off, lens)], out=bad)
    with pytest.raises(ValueError):
        crc32c.batch_multi([(buf, off, lens)], verify=True, mismatch=torch.zeros(2, dtype=torch.uint8, device=dev))
