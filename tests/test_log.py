"""Batched log-record checking (prismdb_amd.log) against the reference log::Reader.

Pinned by tests/golden/log_cases.*: log files written by the reference
log::Writer and read back by the reference log::Reader (oracle/log_fixture.cc,
db/log_test.cc's scenarios plus seeded damage), with every record
(LastRecordOffset, size, crc32c) and every Reporter::Corruption call.

CPU tests drive the host scan + replay with per-record check results from the
oracle; GPU tests get them from the device (one batch for all files)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLD


@pytest.fixture(scope="session")
def log_cases():
    with open(os.path.join(GOLD, "log_cases.json")) as f:
        meta = json.load(f)
    blob = np.fromfile(os.path.join(GOLD, "log_cases.bin"), dtype=np.uint8)
    cases = []
    for c in meta["cases"]:
        f = blob[c["offset"]:c["offset"] + c["size"]].copy()
        for pos, v in c["edits"]:
            f[pos] = v
        cases.append((c, f[:c["keep"]].copy()))
    return cases


def _oracle_bad(oracle, f, off, ln):
    bad = np.zeros(len(off), dtype=np.uint8)
    raw = f.tobytes()
    for i, (o, n) in enumerate(zip(off.tolist(), ln.tolist())):
        stored = int.from_bytes(raw[o:o + 4], "little")
        bad[i] = oracle.value(raw[o + 6:o + 7 + n]) != oracle.unmask(stored)
    return bad


def _check(case, res, oracle):
    want = case["records"]
    got = [[o, len(r), oracle.value(r)] for o, r in zip(res.offsets, res.records)]
    assert got == want, case["name"]
    assert [list(d) for d in res.drops] == case["drops"], case["name"]


def test_log_cases_cover_every_reader_path(log_cases):
    reasons = {m.split("(")[0] for c, _ in log_cases for _, m in c["drops"]}
    assert reasons >= {"Corruption: checksum mismatch", "Corruption: bad record length",
                       "Corruption: partial record without end", "Corruption: missing start of fragmented record",
                       "Corruption: error in middle of record"}
    assert any(m.startswith("Corruption: unknown record type") for c, _ in log_cases for _, m in c["drops"])
    assert sum(len(c["records"]) for c, _ in log_cases) > 20000


def test_replay_matches_reference_reader(native, oracle, log_cases):
    from prismdb_amd import log

    for case, f in log_cases:
        off, ln = log.scan(f, case["initial_offset"])
        bad = _oracle_bad(oracle, f, off, ln) if case["checksum"] else None
        res = log.replay(f, off, ln, bad, checksum=case["checksum"], initial_offset=case["initial_offset"])
        _check(case, res, oracle)


def test_reason_texts(native):
    from prismdb_amd import log

    assert log.reason_text(1) == "Corruption: checksum mismatch"
    assert log.reason_text(256 + 101) == "Corruption: unknown record type 101"
    assert log.reason_text(256 + 0x80) == "Corruption: unknown record type 4294967168"


def test_replay_rejects_foreign_scan(native, log_cases):
    from prismdb_amd import log

    case, f = next((c, f) for c, f in log_cases if c["name"] == "read_write")
    off, ln = log.scan(f)
    with pytest.raises(RuntimeError):
        log.replay(f, off + np.uint64(1), ln, np.zeros(len(off), np.uint8))


@pytest.mark.gpu
def test_read_logs_device_matches_reference_reader(native, oracle, log_cases):
    """Every fixture log through ONE host-resident device batch."""
    from prismdb_amd import log

    res = log.read_logs([f for _, f in log_cases], checksum=True,
                        initial_offsets=[c["initial_offset"] for c, _ in log_cases])
    for (case, f), r in zip(log_cases, res):
        if case["checksum"]:
            _check(case, r, oracle)
    unchecked = [(c, f) for c, f in log_cases if not c["checksum"]]
    res = log.read_logs([f for _, f in unchecked], checksum=False,
                        initial_offsets=[c["initial_offset"] for c, _ in unchecked])
    for (case, f), r in zip(unchecked, res):
        _check(case, r, oracle)


@pytest.mark.gpu
def test_device_resident_log_verify(native, oracle, log_cases):
    """leveldb_crc32c_batch with verify + LOG_HEADER on a device buffer."""
    import torch
    from prismdb_amd import crc32c, log

    dev = torch.device("cuda", 0)
    for case, f in log_cases:
        off, ln = log.scan(f, case["initial_offset"])
        if len(off) == 0:
            continue
        buf = torch.from_numpy(f.copy()).to(dev)
        d_off = torch.from_numpy((off + 6).astype(np.int64)).to(dev)
        d_len = torch.from_numpy((ln + 1).astype(np.int32)).to(dev)
        crc, mm = crc32c.batch(buf, d_off, d_len, verify=True, log_header=True)
        assert (mm.cpu().numpy() == _oracle_bad(oracle, f, off, ln)).all(), case["name"]
        raw = f.tobytes()
        want = [oracle.value(raw[o + 6:o + 7 + n]) for o, n in zip(off.tolist(), ln.tolist())]
        assert crc32c.as_u32(crc) == want, case["name"]


@pytest.mark.gpu
def test_seal_log_reproduces_writer_headers(native, log_cases):
    """Zero every header crc of reference-written logs; one device call reseals
    them byte-identical to what log::Writer wrote."""
    import torch
    from prismdb_amd import log

    dev = torch.device("cuda", 0)
    for name in ("read_write", "many_blocks", "fragmentation", "marginal_trailer", "short_trailer",
                 "random_read", "open_for_append"):
        case, f = next((c, f) for c, f in log_cases if c["name"] == name)
        off, ln = log.scan(f)
        g = f.copy()
        for o in off.tolist():
            g[o:o + 4] = 0
        buf = torch.from_numpy(g).to(dev)
        log.seal_log(buf, torch.from_numpy(off.astype(np.int64)).to(dev),
                     torch.from_numpy(ln.astype(np.int32)).to(dev))
        torch.cuda.synchronize()
        assert (buf.cpu().numpy() == f).all(), name


@pytest.mark.gpu
@pytest.mark.parametrize("with_out", [False, True])
def test_seal_log_without_results(native, log_cases, with_out):
    """The C ABI with out = NULL (and with it): every header crc resealed
    byte-identical, log records of all lengths (the lane kernel's and the
    generic path's) in one call; the lane kernel's results reach the header
    stores through the workspace when the caller keeps none."""
    import ctypes

    import torch
    from prismdb_amd import crc32c, log

    dev = torch.device("cuda", 0)
    cases = [(c, f) for c, f in log_cases if c["name"] in ("read_write", "many_blocks", "fragmentation",
                                                             "marginal_trailer", "random_read")]
    imgs, offs, lens, at = [], [], [], 0
    for _, f in cases:
        off, ln = log.scan(f)
        imgs.append(f)
        offs.append(off.astype(np.int64) + at + 6)  # type || payload
        lens.append(ln.astype(np.int64) + 1)
        at += len(f)
    whole = np.concatenate(imgs)
    g = whole.copy()
    for o in np.concatenate(offs).tolist():
        g[o - 6:o - 2] = 0
    buf = torch.from_numpy(g).to(dev)
    d_off = torch.from_numpy(np.concatenate(offs)).to(dev)
    d_len = torch.from_numpy(np.concatenate(lens).astype(np.int32)).to(dev)
    n = d_off.numel()
    out = torch.empty(n, dtype=torch.int32, device=dev) if with_out else None
    flags = crc32c.FLAG_MASK | crc32c.FLAG_WRITE_TRAILER | crc32c.FLAG_LOG_HEADER
    rc = native.leveldb_crc32c_batch(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, n,
                                     out.data_ptr() if with_out else None, None, flags,
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    assert (buf.cpu().numpy() == whole).all()
    if with_out:
        stored = whole[(np.concatenate(offs) - 6)[:, None] + np.arange(4)[None, :]].reshape(-1).view("<u4")
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), stored)
