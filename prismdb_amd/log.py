"""Batched log (WAL / MANIFEST) record checking.

PrismDB recovers its write-ahead logs and MANIFEST through LevelDB's
log::Reader (db/log_reader.cc), which checks one physical record at a time:
crc32c(type || payload) against the record header (db/log_reader.cc:245-258).
Here every record of one or many log files is checked in one device batch and
the reader's control flow is replayed over the answers, so the result is what
the reference reader returns, record for record and drop for drop:

    read_log(image, checksum=True, initial_offset=0) -> LogReadResult
    read_logs([image, ...])                            one device pass for all files
    seal_log(buf, header_off, length)                  log::Writer's header crc
                                                       (db/log_writer.cc:90-97)
                                                       for many records, in place

Host side: include/prismdb_log.h (prismdb_amd/csrc/log_reader.cc).  Device
side: leveldb_crc32c_batch_host / leveldb_crc32c_batch with
PRISMDB_CRC32C_LOG_HEADER.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from . import crc32c
from ._lib import lib

BLOCK_SIZE = 32768  # db/log_format.h
HEADER_SIZE = 7
FULL, FIRST, MIDDLE, LAST = 1, 2, 3, 4
ECAPACITY = -11


class _ReplayOut(ctypes.Structure):
    _fields_ = [
        ("record_offset", ctypes.c_void_p), ("record_first", ctypes.c_void_p), ("record_nfrag", ctypes.c_void_p),
        ("record_cap", ctypes.c_size_t), ("n_records", ctypes.c_size_t),
        ("fragment", ctypes.c_void_p), ("fragment_cap", ctypes.c_size_t), ("n_fragments", ctypes.c_size_t),
        ("drop_bytes", ctypes.c_void_p), ("drop_reason", ctypes.c_void_p),
        ("drop_cap", ctypes.c_size_t), ("n_drops", ctypes.c_size_t),
    ]


def _log_lib():
    L = lib()
    if not hasattr(L, "_log_declared"):
        sz, vp, u64 = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint64
        L.leveldb_log_scan.restype = ctypes.c_int
        L.leveldb_log_scan.argtypes = [vp, sz, u64, vp, vp, sz, ctypes.POINTER(sz)]
        L.leveldb_log_replay.restype = ctypes.c_int
        L.leveldb_log_replay.argtypes = [vp, sz, u64, ctypes.c_int, vp, vp, vp, sz, ctypes.POINTER(_ReplayOut)]
        L.leveldb_log_reason.restype = ctypes.c_char_p
        L.leveldb_log_reason.argtypes = [ctypes.c_int32, ctypes.c_char_p, sz]
        L._log_declared = True
    return L


def _as_u8(image):
    import numpy as np

    if isinstance(image, np.ndarray):
        return np.ascontiguousarray(image, dtype=np.uint8)
    return np.frombuffer(bytes(image), dtype=np.uint8)


def reason_text(code: int) -> str:
    """Status::Corruption(reason).ToString() for a drop reason code."""
    buf = ctypes.create_string_buffer(96)
    return _log_lib().leveldb_log_reason(code, buf, len(buf)).decode()


def scan(image, initial_offset: int = 0):
    """(header_off uint64[n], length uint32[n]) of every physical record log::Reader can reach."""
    import numpy as np

    f = _as_u8(image)
    L = _log_lib()
    cap = len(f) // HEADER_SIZE + 1
    off = np.empty(cap, dtype=np.uint64)
    ln = np.empty(cap, dtype=np.uint32)
    n = ctypes.c_size_t(0)
    rc = L.leveldb_log_scan(f.ctypes.data, len(f), initial_offset, off.ctypes.data, ln.ctypes.data, cap,
                            ctypes.byref(n))
    if rc != 0:
        raise RuntimeError(f"leveldb_log_scan failed ({rc})")
    return off[:n.value], ln[:n.value]


@dataclass
class LogReadResult:
    """What log::Reader::ReadRecord returns until EOF, plus the Reporter calls."""
    records: List[bytes] = field(default_factory=list)
    offsets: List[int] = field(default_factory=list)            # LastRecordOffset() per record
    drops: List[Tuple[int, str]] = field(default_factory=list)  # Reporter::Corruption(bytes, status)

    @property
    def dropped_bytes(self) -> int:
        return sum(b for b, _ in self.drops)


def replay(image, off, ln, bad, *, checksum: bool = True, initial_offset: int = 0) -> LogReadResult:
    """Run the reader's state machine over a scan and per-record check results."""
    import numpy as np

    f = _as_u8(image)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    n = len(off)
    bad_arr = np.ascontiguousarray(bad, dtype=np.uint8) if bad is not None else None
    rec_off = np.empty(n, dtype=np.uint64)
    rec_first = np.empty(n, dtype=np.uint32)
    rec_nfrag = np.empty(n, dtype=np.uint32)
    frag = np.empty(n, dtype=np.uint32)
    dcap = 2 * (n + len(f) // BLOCK_SIZE + 2)
    dbytes = np.empty(dcap, dtype=np.uint64)
    dreason = np.empty(dcap, dtype=np.int32)
    out = _ReplayOut(rec_off.ctypes.data, rec_first.ctypes.data, rec_nfrag.ctypes.data, n, 0,
                     frag.ctypes.data, n, 0, dbytes.ctypes.data, dreason.ctypes.data, dcap, 0)
    rc = _log_lib().leveldb_log_replay(f.ctypes.data, len(f), initial_offset, 1 if checksum else 0,
                                       off.ctypes.data if n else None, ln.ctypes.data if n else None,
                                       bad_arr.ctypes.data if bad_arr is not None and n else None, n,
                                       ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(f"leveldb_log_replay failed ({rc})")
    res = LogReadResult()
    raw = f.tobytes()
    for r in range(out.n_records):
        parts = []
        for q in range(int(rec_first[r]), int(rec_first[r]) + int(rec_nfrag[r])):
            k = int(frag[q])
            s = int(off[k]) + HEADER_SIZE
            parts.append(raw[s:s + int(ln[k])])
        res.records.append(b"".join(parts))
        res.offsets.append(int(rec_off[r]))
    res.drops = [(int(dbytes[i]), reason_text(int(dreason[i]))) for i in range(out.n_drops)]
    return res


def read_logs(images: Sequence, *, checksum: bool = True,
              initial_offsets: Optional[Sequence[int]] = None) -> List[LogReadResult]:
    """log::Reader over many log images, every record checked in ONE device batch.

    The images are packed into one host buffer and streamed through the device
    by leveldb_crc32c_batch_host (verify with PRISMDB_CRC32C_LOG_HEADER);
    the replay then runs per file on the host."""
    import numpy as np

    imgs = [_as_u8(im) for im in images]
    inits = list(initial_offsets) if initial_offsets is not None else [0] * len(imgs)
    scans, bases = [], []
    base = 0
    for im, io in zip(imgs, inits):
        scans.append(scan(im, io))
        bases.append(base)
        base += len(im)
    bad_all = None
    n_all = sum(len(s[0]) for s in scans)
    if checksum and n_all:
        blob = np.empty(base, dtype=np.uint8)
        for im, b in zip(imgs, bases):
            blob[b:b + len(im)] = im
        span_off = np.concatenate([s[0] + np.uint64(b + 6) for s, b in zip(scans, bases)])
        span_len = np.concatenate([s[1] + np.uint32(1) for s in scans])
        _, bad_all = crc32c.batch_host(blob, span_off, span_len, verify=True, log_header=True)
    results, at = [], 0
    for im, io, (o, ln) in zip(imgs, inits, scans):
        bad = bad_all[at:at + len(o)] if bad_all is not None else None
        at += len(o)
        results.append(replay(im, o, ln, bad, checksum=checksum, initial_offset=io))
    return results


def read_log(image, *, checksum: bool = True, initial_offset: int = 0) -> LogReadResult:
    return read_logs([image], checksum=checksum, initial_offsets=[initial_offset])[0]


def seal_log(buf, header_off, length, *, stream=None, check_bounds: bool = True):
    """Write log::Writer's header checksum (db/log_writer.cc:90-97) in place.

    buf: device uint8 tensor of log blocks whose physical records have their
    length and type bytes filled in; header_off (int64) / length (int32) name
    the records.  Bytes [h, h+4) of each header get Mask(crc32c(type ||
    payload)).  Returns the masked CRCs (int32).  Everything runs on `stream`
    (default: torch's current stream)."""
    import torch
    from contextlib import nullcontext

    with torch.cuda.stream(stream) if stream is not None else nullcontext():
        span_off = header_off + 6
        span_len = length + 1
        out, _ = crc32c.batch(buf, span_off, span_len, mask=True, trailer=True, log_header=True,
                              check_bounds=check_bounds)
    return out
