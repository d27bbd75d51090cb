"""The link-time drop-in: the reference's own SST and log code
-- table/table_builder.cc (WriteRawBlock: Mask(Value(contents||type)),
table/table_builder.cc:185-202), table/format.cc (ReadBlock verify,
table/format.cc:91-102), db/log_writer.cc and db/log_reader.cc (record crcs,
db/log_writer.cc:94-95, db/log_reader.cc:247-248) -- compiled UNCHANGED from
/root/reference against this repository's include/util/crc32c.h, with
util/crc32c.cc left out and leveldb::crc32c::Extend linked from
libprismdb_crc32c.so (oracle/Makefile target `dropin`).  The SST it writes
(and re-reads with verify_checksums and paranoid_checks) and the 107 log
files it writes and reads back must be byte-identical to the pure-reference
build's.  CPU only; skipped where /root/reference is absent (the GPU box)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "oracle", "_ref")
EXTEND = "_ZN7leveldb6crc32c6ExtendEjPKcm"

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "util")),
                                reason="needs the reference sources (/root/reference)")


@pytest.fixture(scope="module")
def built(native):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref", "dropin"])
    return OUT


def _nm(args):
    return subprocess.run(["nm"] + args, capture_output=True, text=True, check=True).stdout


def test_extend_comes_from_the_product_library(built):
    """The drop-in objects define no Extend; the binaries import it, and the
    product library exports it (the pure-reference build defines its own)."""
    objs = []
    for d, _, files in os.walk(os.path.join(built, "dropin")):
        objs += [os.path.join(d, f) for f in files if f.endswith(".o")]
    assert any(o.endswith("table_builder.o") for o in objs) and any(o.endswith("log_writer.o") for o in objs)
    assert not any(o.endswith(os.path.join("util", "crc32c.o")) for o in objs)
    defined = _nm(["--defined-only"] + objs)
    assert EXTEND not in defined
    undefined = _nm(["--undefined-only"] + objs)
    assert EXTEND in undefined  # format.o, table_builder.o, log_*.o call it
    for exe in ("sst_fixture_dropin", "log_fixture_dropin"):
        assert EXTEND in _nm(["-D", "--undefined-only", os.path.join(built, exe)])
        ldd = subprocess.run(["ldd", os.path.join(built, exe)], capture_output=True, text=True).stdout
        assert "libprismdb_crc32c.so" in ldd
    lib = os.path.join(ROOT, "prismdb_amd", "lib", "libprismdb_crc32c.so")
    assert f"T {EXTEND}" in _nm(["-D", "--defined-only", lib])
    assert f"T {EXTEND}" in _nm(["--defined-only", os.path.join(built, "sst_fixture")])


@pytest.mark.parametrize("nkeys,value_len,block_size", [(3000, 980, 4096), (500, 100, 1024), (64, 4000, 16384)])
def test_sst_byte_identical(built, tmp_path, nkeys, value_len, block_size):
    """TableBuilder -> file -> Table::Open (paranoid) -> full iteration with
    verify_checksums, through the reference code linked to our Extend."""
    outs = {}
    for exe in ("sst_fixture", "sst_fixture_dropin"):
        ldb, js = tmp_path / f"{exe}.ldb", tmp_path / f"{exe}.json"
        r = subprocess.run([os.path.join(built, exe), str(ldb), str(js), str(nkeys), str(value_len),
                            str(block_size)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        assert f"verified {nkeys} keys" in r.stdout
        outs[exe] = (ldb.read_bytes(), js.read_bytes())
    assert outs["sst_fixture"] == outs["sst_fixture_dropin"]


def test_log_byte_identical(built, tmp_path):
    """log::Writer -> log::Reader over the 107 reference log scenarios
    (db/log_test.cc's cases and seeded damage): the records, the corruption
    reports and the files written are identical."""
    outs = {}
    for exe in ("log_fixture", "log_fixture_dropin"):
        prefix = tmp_path / exe
        r = subprocess.run([os.path.join(built, exe), str(prefix)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[exe] = ((tmp_path / f"{exe}.bin").read_bytes(), (tmp_path / f"{exe}.json").read_bytes())
    assert outs["log_fixture"] == outs["log_fixture_dropin"]
