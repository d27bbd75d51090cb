"""Shared fixtures.  `-m gpu` tests need a real MI355X; everything else runs on CPU.

The oracle (oracle/crc32c_oracle.c, built to oracle/_build/liboracle.so) is the
parity checker; tests are the only product-adjacent code allowed to load it.
"""
import ctypes
import json
import os
import subprocess

import pytest

# The library's prismdb_* routing and fault-injection setters act only in a
# process started with this (crc32c_capi.hip, TestHooksEnabled); the tests pin
# routes with them.  Set before the library's first hook call.
os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


class Oracle:
    """ctypes face of oracle/crc32c_oracle.c."""

    def __init__(self, path):
        self.lib = ctypes.CDLL(path)
        u8p = ctypes.c_void_p
        L = self.lib
        L.oracle_crc32c_extend.restype = ctypes.c_uint32
        L.oracle_crc32c_extend.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.oracle_crc32c_extend_bitwise.restype = ctypes.c_uint32
        L.oracle_crc32c_extend_bitwise.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.oracle_crc32c_mask.restype = ctypes.c_uint32
        L.oracle_crc32c_mask.argtypes = [ctypes.c_uint32]
        L.oracle_crc32c_unmask.restype = ctypes.c_uint32
        L.oracle_crc32c_unmask.argtypes = [ctypes.c_uint32]
        L.oracle_crc32c_batch.restype = ctypes.c_size_t
        L.oracle_crc32c_batch.argtypes = [u8p, u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_uint32, u8p]
        L.oracle_crc32c_batch_fixed.restype = None
        L.oracle_crc32c_batch_fixed.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                ctypes.c_uint32, u8p, ctypes.c_uint32]
        L.oracle_fill_synthetic.restype = None
        L.oracle_fill_synthetic.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]

    @staticmethod
    def _ptr(b):
        import numpy as np

        if isinstance(b, np.ndarray):
            return b.ctypes.data
        return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value

    def extend(self, init, data: bytes) -> int:
        return self.lib.oracle_crc32c_extend(init, data, len(data))

    def extend_bitwise(self, init, data: bytes) -> int:
        return self.lib.oracle_crc32c_extend_bitwise(init, data, len(data))

    def value(self, data: bytes) -> int:
        return self.extend(0, data)

    def mask(self, c):
        return self.lib.oracle_crc32c_mask(c)

    def unmask(self, c):
        return self.lib.oracle_crc32c_unmask(c)

    def synth(self, nbytes, seed, byte_offset=0):
        import numpy as np

        a = np.empty(nbytes, dtype=np.uint8)
        self.lib.oracle_fill_synthetic(a.ctypes.data, nbytes, seed, byte_offset)
        return a

    def batch(self, buf, off, lens, init=None, mask=False, verify=False):
        """numpy in/out; returns (crc uint32[n], mismatch uint8[n] or None)."""
        import numpy as np

        n = len(off)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.empty(n, dtype=np.uint32)
        mm = np.empty(n, dtype=np.uint8) if verify else None
        ini = np.ascontiguousarray(init, dtype=np.uint32) if init is not None else None
        self.lib.oracle_crc32c_batch(buf.ctypes.data, off.ctypes.data, lens.ctypes.data,
                                     ini.ctypes.data if ini is not None else None, n, out.ctypes.data,
                                     1 if mask else 0, mm.ctypes.data if verify else None)
        return out, mm

    def batch_fixed(self, buf, stride, length, nblocks, init=0, mask=False):
        import numpy as np

        out = np.empty(nblocks, dtype=np.uint32)
        self.lib.oracle_crc32c_batch_fixed(buf.ctypes.data, stride, length, nblocks, init, out.ctypes.data,
                                           1 if mask else 0)
        return out


@pytest.fixture(scope="session")
def oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"])
    return Oracle(ORACLE_SO)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLD, "kat.json")) as f:
        kat = json.load(f)
    with open(os.path.join(GOLD, "crc32c_vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(GOLD, vec["input"]), "rb") as f:
        inp = f.read()
    with open(os.path.join(GOLD, "stream_vectors.json")) as f:
        stream = json.load(f)
    with open(os.path.join(GOLD, "sst_small.json")) as f:
        sst = json.load(f)
    with open(os.path.join(GOLD, "sst_small.ldb"), "rb") as f:
        sst_bytes = f.read()
    return {"kat": kat, "vectors": vec, "input": inp, "stream": stream, "sst": sst, "sst_bytes": sst_bytes}


@pytest.fixture(scope="session")
def native():
    """The product native library (built by __graft_entry__.build / prismdb_amd.build)."""
    from prismdb_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        from prismdb_amd.build import build

        build()
    return _lib.lib()


# Descriptor-batch routes the GPU tests pin (C-ABI test hooks, not public):
#   direct     the one-launch kernel (crc32c_direct.hip; the default for
#              batches of <= 2^17 spans) and, pinned here, windows of 2^17
#              spans back to back for larger ones (log-record batches aside;
#              the default: windows up to 2^18 spans, the planner beyond)
#   windows    the one-launch kernel in windows of 1000 spans (many windows
#              on modest batches)
#   lane_log   the planner path, lane kernel in front of log-record batches
#              (the default for log-record batches of > 2^17 spans)
#   lane_all   the planner path, lane kernel in front of every batch
#   span_only  the planner path alone
ROUTES = {"direct": (1 << 17, 0), "windows": (1000, 0), "lane_log": (0, 0), "lane_all": (0, 1),
          "span_only": (0, -1)}


def set_route(native, name):
    """Pin a route; returns a callable restoring the defaults."""
    direct_max, lane = ROUTES[name]
    native.prismdb_crc32c_direct_max(direct_max)
    native.prismdb_crc32c_lane_mode(lane)
    native.prismdb_crc32c_windows(1 if name in ("direct", "windows") else 0)

    def restore():
        native.prismdb_crc32c_direct_max(1 << 17)
        native.prismdb_crc32c_lane_mode(0)
        native.prismdb_crc32c_windows(2)

    return restore


@pytest.fixture(params=["direct", "windows", "lane_log"])
def route(request, native):
    """The default descriptor routes: one-launch (one launch or windows) and planner."""
    restore = set_route(native, request.param)
    yield request.param
    restore()


@pytest.fixture(params=list(ROUTES))
def any_route(request, native):
    """Every descriptor route."""
    restore = set_route(native, request.param)
    yield request.param
    restore()


@pytest.fixture(params=["windows", "planner"])
def bulk_route(request, native):
    """Batches of more than 2^17 spans: windows of the one-launch kernel and
    the planner path (the default picks windows up to 2^18 spans)."""
    prev = native.prismdb_crc32c_windows(1 if request.param == "windows" else 0)
    yield request.param
    native.prismdb_crc32c_windows(prev)


@pytest.fixture
def planner_bulk(native):
    """Pin the planner path for batches of more than 2^17 spans (tests of its
    own machinery: pair runs, slices, the segment workspace)."""
    prev = native.prismdb_crc32c_windows(0)
    yield "planner"
    native.prismdb_crc32c_windows(prev)
