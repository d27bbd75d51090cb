"""Argument checking of the batch C ABI (include/prismdb_crc32c.h), on CPU.

Every entry point validates its arguments before it touches a device, so
these run without a GPU: bad arguments give PRISMDB_CRC32C_EINVAL (-1) and a
thread-local message, an empty batch is a no-op, and -- where no device is
present -- a valid call fails loudly with PRISMDB_CRC32C_EDEVICE (-2)
instead of falling back to the CPU.  The reference has no such surface (its
Extend cannot fail, util/crc32c.h:17); the caller maps a mismatch flag, not
an error, to Status::Corruption (table/format.cc:99)."""
import ctypes

import numpy as np
import pytest

EINVAL, EDEVICE = -1, -2
MASK, WRITE_TRAILER, LOG_HEADER = 0x1, 0x2, 0x4


def _err(native):
    return native.leveldb_crc32c_last_error().decode()


@pytest.fixture()
def bufs():
    data = np.zeros(1 << 16, dtype=np.uint8)
    off = np.arange(4, dtype=np.uint64) * 4096
    ln = np.full(4, 4000, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    mm = np.zeros(4, dtype=np.uint8)
    return data, off, ln, out, mm


def test_empty_batches_are_noops(native, bufs):
    data, off, ln, out, _ = bufs
    assert native.leveldb_crc32c_batch(None, None, None, None, 0, None, None, 0, None) == 0
    assert native.leveldb_crc32c_batch_fixed(None, 4096, 4096, 0, 0, None, None, 0, None) == 0
    assert native.leveldb_crc32c_batch_host(None, None, None, None, 0, None, None, 0) == 0


def test_batch_rejects_null_descriptors(native, bufs):
    data, off, ln, out, _ = bufs
    rc = native.leveldb_crc32c_batch(data.ctypes.data, None, ln.ctypes.data, None, 4, out.ctypes.data, None, 0,
                                     None)
    assert rc == EINVAL and "non-NULL" in _err(native)
    rc = native.leveldb_crc32c_batch_fixed(None, 4096, 4096, 4, 0, out.ctypes.data, None, 0, None)
    assert rc == EINVAL and "dev_base" in _err(native)


@pytest.mark.parametrize("flags", [0x10, 0x100, 0xFFFFFFF0])
def test_unknown_flag_bits(native, bufs, flags):
    data, off, ln, out, _ = bufs
    rc = native.leveldb_crc32c_batch(data.ctypes.data, off.ctypes.data, ln.ctypes.data, None, 4, out.ctypes.data,
                                     None, flags, None)
    assert rc == EINVAL and "flag" in _err(native)
    rc = native.leveldb_crc32c_batch_fixed(data.ctypes.data, 4096, 4000, 4, 0, out.ctypes.data, None, flags, None)
    assert rc == EINVAL and "flag" in _err(native)


def test_trailer_and_verify_are_exclusive(native, bufs):
    data, off, ln, out, mm = bufs
    rc = native.leveldb_crc32c_batch(data.ctypes.data, off.ctypes.data, ln.ctypes.data, None, 4, out.ctypes.data,
                                     mm.ctypes.data, WRITE_TRAILER, None)
    assert rc == EINVAL and "exclusive" in _err(native)


def test_fixed_length_limit(native, bufs):
    data, _, _, out, _ = bufs
    rc = native.leveldb_crc32c_batch_fixed(data.ctypes.data, 1 << 33, 1 << 32, 1, 0, out.ctypes.data, None, 0,
                                           None)
    assert rc == EINVAL and "4 GiB" in _err(native)


def test_host_batch_checks(native, bufs):
    data, off, ln, out, mm = bufs
    p = data.ctypes.data
    assert native.leveldb_crc32c_batch_host(p, off.ctypes.data, ln.ctypes.data, None, 4, out.ctypes.data, None,
                                            0x8) == EINVAL  # UNORDERED: device batches only
    assert "MASK" in _err(native)
    # WRITE_TRAILER seals host buffers, but not while verifying
    assert native.leveldb_crc32c_batch_host(p, off.ctypes.data, ln.ctypes.data, None, 4, out.ctypes.data,
                                            mm.ctypes.data, WRITE_TRAILER) == EINVAL
    assert "exclusive" in _err(native)
    # a log-record seal writes 6 bytes before each span
    off2 = np.array([3, 4096], dtype=np.uint64)
    assert native.leveldb_crc32c_batch_host(p, off2.ctypes.data, ln.ctypes.data, None, 2, out.ctypes.data, None,
                                            WRITE_TRAILER | LOG_HEADER) == EINVAL
    assert "header" in _err(native)
    unsorted = off[::-1].copy()
    assert native.leveldb_crc32c_batch_host(p, unsorted.ctypes.data, ln.ctypes.data, None, 4, out.ctypes.data,
                                            None, 0) == EINVAL
    assert "sorted" in _err(native)
    big = np.full(4, (64 << 20) + 1, dtype=np.uint32)
    assert native.leveldb_crc32c_batch_host(p, off.ctypes.data, big.ctypes.data, None, 4, out.ctypes.data, None,
                                            0) == EINVAL
    assert "64 MiB" in _err(native)
    # verify with LOG_HEADER reads 6 bytes before each span: the first may not start before byte 6
    off0 = np.array([2, 4096], dtype=np.uint64)
    assert native.leveldb_crc32c_batch_host(p, off0.ctypes.data, ln.ctypes.data, None, 2, out.ctypes.data,
                                            mm.ctypes.data, LOG_HEADER) == EINVAL
    assert "header" in _err(native)


def test_no_device_fails_loudly(native, bufs):
    """Without a HIP device a valid call returns EDEVICE and says why; there is
    no CPU fallback behind the batch entry points."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    data, off, ln, out, _ = bufs
    rc = native.leveldb_crc32c_batch(data.ctypes.data, off.ctypes.data, ln.ctypes.data, None, 4, out.ctypes.data,
                                     None, 0, None)
    assert rc == EDEVICE, (rc, _err(native))
    assert _err(native)
    assert native.leveldb_crc32c_batch_fixed(data.ctypes.data, 4096, 4000, 4, 0, out.ctypes.data, None, 0,
                                             None) == EDEVICE
    assert native.leveldb_crc32c_device_init(ctypes.c_int(0)) == EDEVICE


def test_python_host_batch_bounds(native):
    """prismdb_amd.crc32c.batch_host checks descriptors against the host buffer
    before calling the engine: spans (with their stored trailer or log header)
    inside the buffer, equal-length descriptor arrays."""
    from prismdb_amd import crc32c

    data = np.zeros(8192, dtype=np.uint8)
    off = np.array([0, 4096], dtype=np.uint64)
    with pytest.raises(ValueError, match="outside"):
        crc32c.batch_host(data, off, np.array([4096, 4097], dtype=np.uint32))
    with pytest.raises(ValueError, match="outside"):  # the verify trailer of the last span
        crc32c.batch_host(data, off, np.array([4000, 4093], dtype=np.uint32), verify=True)
    with pytest.raises(ValueError, match="outside"):  # the log header before the first span
        crc32c.batch_host(data, np.array([3, 100], dtype=np.uint64), np.array([10, 10], dtype=np.uint32),
                          verify=True, log_header=True)
    with pytest.raises(ValueError, match="same length"):
        crc32c.batch_host(data, off, np.array([10], dtype=np.uint32))
    with pytest.raises(ValueError, match="same length"):
        crc32c.batch_host(data, off, np.array([10, 10], dtype=np.uint32), init=np.array([1], dtype=np.uint32))


def test_host_seal_rejects_read_only_memory(native):
    """WRITE_TRAILER into a PROT_READ mapping returns EINVAL (the C side probes
    the first and last trailer slots before the call stores anything) instead
    of faulting in the trailer stores; the same spans without WRITE_TRAILER
    get past that check (and, without a device, fail with EDEVICE)."""
    import mmap

    import torch

    m = mmap.mmap(-1, 3 * 4096, prot=mmap.PROT_READ)
    ro = np.frombuffer(m, dtype=np.uint8)
    addr = ro.ctypes.data
    off = np.array([0, 4096], dtype=np.uint64)
    ln = np.array([4000, 4000], dtype=np.uint32)
    out = np.zeros(2, dtype=np.uint32)
    for flags in (WRITE_TRAILER | 1, WRITE_TRAILER | LOG_HEADER):
        o = off + 8 if flags & LOG_HEADER else off
        rc = native.leveldb_crc32c_batch_host(addr, o.ctypes.data, ln.ctypes.data, None, 2, out.ctypes.data,
                                              None, flags)
        assert rc == EINVAL and "not writable" in _err(native), (flags, rc, _err(native))
    # writable memory passes the probe, and the probe leaves its bytes as they were
    rw = np.arange(3 * 4096, dtype=np.uint64).astype(np.uint8)
    before = rw.copy()
    rc = native.leveldb_crc32c_batch_host(rw.ctypes.data, off.ctypes.data, ln.ctypes.data, None, 2,
                                          out.ctypes.data, None, WRITE_TRAILER)
    if not torch.cuda.is_available():
        assert rc == EDEVICE, (rc, _err(native))
        np.testing.assert_array_equal(rw, before)
    del ro
    m.close()


def test_python_host_seal_rejects_read_only_or_strided(native):
    """prismdb_amd.crc32c.batch_host: trailer=True on a read-only array (a
    np.frombuffer view of bytes) or any call on a strided view raises
    ValueError before the engine is called."""
    from prismdb_amd import crc32c

    off = np.array([0, 4096], dtype=np.uint64)
    ln = np.array([4000, 4000], dtype=np.uint32)
    ro = np.frombuffer(bytes(8192), dtype=np.uint8)
    with pytest.raises(ValueError, match="read-only"):
        crc32c.batch_host(ro, off, ln, mask=True, trailer=True)
    strided = np.zeros(2 * 8192, dtype=np.uint8)[::2]
    with pytest.raises(ValueError, match="contiguous"):
        crc32c.batch_host(strided, off, ln)
    with pytest.raises(ValueError, match="contiguous"):
        crc32c.batch_host(strided, off, ln, trailer=True)


def test_python_host_batch_offsets_do_not_wrap(native):
    """A negative offset (-1 would wrap to 2^64 - 1) and an offset past the
    buffer whose end wraps back inside it are rejected, not passed on."""
    from prismdb_amd import crc32c

    data = np.zeros(8192, dtype=np.uint8)
    with pytest.raises(ValueError, match="negative"):
        crc32c.batch_host(data, np.array([-1, 0], dtype=np.int64), np.array([1, 10], dtype=np.uint32))
    wrap = np.array([0, 2**64 - 16], dtype=np.uint64)  # + 32 wraps to 16
    with pytest.raises(ValueError, match="outside"):
        crc32c.batch_host(data, wrap, np.array([10, 32], dtype=np.uint32))


def _multi(native, ndev, devices, base, off, ln, n, out, mm=None, flags=0, init=None):
    P = ctypes.c_void_p * max(ndev, 1)
    return native.leveldb_crc32c_batch_multi(
        ndev, (ctypes.c_int * len(devices))(*devices) if devices is not None else None,
        P(*base) if base is not None else None, P(*off) if off is not None else None,
        P(*ln) if ln is not None else None, P(*init) if init is not None else None,
        (ctypes.c_size_t * len(n))(*n) if n is not None else None, out, mm, flags, None)


def test_multi_argument_checks(native, bufs):
    """leveldb_crc32c_batch_multi checks its arguments before any device or
    RCCL call: device count, NULL arrays, a device listed twice, a
    partition's NULL descriptors, results wanted somewhere, flags."""
    data, off, ln, out, mm = bufs
    b, o, l, po = data.ctypes.data, off.ctypes.data, ln.ctypes.data, out.ctypes.data
    assert _multi(native, 0, [0], [b], [o], [l], [4], po) == EINVAL and "ndev" in _err(native)
    assert _multi(native, 65, [0], [b], [o], [l], [4], po) == EINVAL and "ndev" in _err(native)
    assert _multi(native, 1, None, [b], [o], [l], [4], po) == EINVAL and "non-NULL" in _err(native)
    assert _multi(native, 1, [0], [b], [o], [l], None, po) == EINVAL and "non-NULL" in _err(native)
    assert _multi(native, 2, [0, 0], [b, b], [o, o], [l, l], [4, 4], po) == EINVAL
    assert "twice" in _err(native)
    assert _multi(native, 1, [-1], [b], [o], [l], [4], po) == EINVAL and "negative" in _err(native)
    assert _multi(native, 2, [0, 1], [b, None], [o, o], [l, l], [4, 4], po) == EINVAL
    assert "NULL" in _err(native)
    assert _multi(native, 1, [0], [b], [o], [l], [4], None) == EINVAL and "out0 or mismatch0" in _err(native)
    assert _multi(native, 1, [0], [b], [o], [l], [4], po, flags=0x10) == EINVAL and "flag" in _err(native)
    assert _multi(native, 1, [0], [b], [o], [l], [4], po, mm.ctypes.data, WRITE_TRAILER) == EINVAL
    assert "exclusive" in _err(native)


def test_test_hooks_gated_by_environment():
    """The prismdb_* routing and fault-injection setters are process-global:
    without PRISMDB_ENABLE_TEST_HOOKS=1 they change nothing (a PrismDB
    partition thread cannot reroute or fail the others' batches) and report
    the current setting; with it they act.  Run in fresh processes (the
    switch is read once)."""
    import os
    import subprocess
    import sys

    code = ("import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); L.prismdb_crc32c_direct_max.restype = ctypes.c_uint64; "
            "L.prismdb_crc32c_direct_max.argtypes = [ctypes.c_uint64]; L.prismdb_crc32c_windows.argtypes = [ctypes.c_int]; "
            "a = L.prismdb_crc32c_direct_max(5); b = L.prismdb_crc32c_direct_max(7); "
            "w = L.prismdb_crc32c_windows(0); w2 = L.prismdb_crc32c_windows(1); "
            "print(L.prismdb_test_hooks_enabled(), a, b, w, w2)")
    from prismdb_amd import _lib

    for flag, want in ((None, "0 131072 131072 2 2"), ("1", "1 131072 5 2 0")):
        env = {k: v for k, v in os.environ.items() if k != "PRISMDB_ENABLE_TEST_HOOKS"}
        if flag:
            env["PRISMDB_ENABLE_TEST_HOOKS"] = flag
        r = subprocess.run([sys.executable, "-c", code, _lib.LIB_PATH], env=env, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert r.stdout.strip() == want, (flag, r.stdout, r.stderr)
