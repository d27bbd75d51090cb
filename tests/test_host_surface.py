"""The per-call host surface (leveldb::crc32c::Extend and the C ABI) and the
exported symbol set of the native library.  No GPU needed: nothing here
launches a kernel."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT


def _declared_symbols():
    names = set()
    for h in ("prismdb_crc32c.h", "prismdb_synth.h", "prismdb_sst.h", "prismdb_log.h"):
        with open(os.path.join(ROOT, "include", h)) as f:
            src = f.read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*([a-z_0-9]+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol(native):
    from prismdb_amd import _lib

    declared = _declared_symbols()
    assert set(_lib.C_ABI_SYMBOLS) == declared
    for name in declared:
        assert hasattr(native, name), name
    # the C++ drop-in: leveldb::crc32c::Extend(unsigned, const char*, unsigned long)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert _lib.CXX_EXTEND_SYMBOL in out
    for name in declared:
        assert re.search(rf"\bT {name}\b", out), name


def test_host_extend_kats(native, golden):
    from prismdb_amd import crc32c

    kat = golden["kat"]
    for v in kat["vectors"]:
        data = bytes.fromhex(v["hex"])
        assert crc32c.Value(data) == v["value"], v["name"]
        assert crc32c.Mask(v["value"]) == v["masked"]
        assert crc32c.Unmask(v["masked"]) == v["value"]
    assert crc32c.Extend(crc32c.Value("hello "), "world") == crc32c.Value("hello world")
    assert crc32c.Value("TestCRCBuffer") == 0xDCBC59FA


@pytest.mark.parametrize("portable", [False, True])
def test_host_extend_sweep(native, golden, portable):
    inp = golden["input"]
    fn = native.prismdb_crc32c_extend_portable if portable else native.leveldb_crc32c_extend
    for off, n, init, crc, _ in golden["vectors"]["rows"]:
        buf = ctypes.create_string_buffer(inp[off:off + n], n)
        # also exercise every buffer alignment of the host paths
        assert fn(init, ctypes.cast(buf, ctypes.c_char_p), n) == crc, (off, n, init)


def test_combine(native, golden):
    from prismdb_amd import crc32c

    inp = golden["input"]
    for cut in (0, 1, 3, 100, 4096, 40000):
        a, b = inp[:cut], inp[cut:70000]
        assert crc32c.Combine(crc32c.Value(a), crc32c.Value(b), len(b)) == crc32c.Value(inp[:70000])


def test_accelerated_flag_is_consistent(native):
    from prismdb_amd import crc32c

    assert crc32c.accelerated() in (True, False)
