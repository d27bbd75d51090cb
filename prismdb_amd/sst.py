"""Whole-SST batch checksumming on the MI355X engine.

verify_tables(images)   ReadBlock's verify (table/format.cc:91-102) for every
                        block of one or more SST images in ONE device batch;
                        per block "OK" or "Corruption: block checksum mismatch".
seal_blocks(buf, ...)   TableBuilder::WriteRawBlock's trailer
                        (table/table_builder.cc:185-202) for many blocks at
                        once, written in place on the device.

The SST layout is walked on the host by the native library
(include/prismdb_sst.h, prismdb_amd/csrc/sst.cc); the checksums run on the
device through leveldb_crc32c_batch.
"""
from __future__ import annotations

import ctypes
from contextlib import nullcontext
from dataclasses import dataclass
from typing import List, Sequence

from . import crc32c
from ._lib import lib

KIND_NAMES = {0: "data", 1: "filter", 2: "metaindex", 3: "index"}
SST_ECORRUPT = -10
SST_ECAPACITY = -11
SST_EUNSUPPORTED = -12
OK = "OK"
MISMATCH = "Corruption: block checksum mismatch"  # table/format.cc:99


class SstError(Exception):
    """A table whose blocks cannot be listed; str() is the reference's Status text."""


class SstCorruption(SstError):
    """Status::Corruption raised while walking the table layout."""


class SstUnsupported(SstError):
    """Status::NotSupported: a snappy-compressed index or metaindex block
    (the walker does not decompress; include/prismdb_sst.h)."""


def _raise(rc: int, msg: str):
    raise (SstUnsupported if rc == SST_EUNSUPPORTED else SstCorruption)(msg)


def _sst_lib():
    L = lib()
    if not hasattr(L, "_sst_declared"):
        L.leveldb_sst_block_spans.restype = ctypes.c_int
        L.leveldb_sst_block_spans.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.leveldb_sst_last_error.restype = ctypes.c_char_p
        L._sst_declared = True
    return L


def block_spans(image: bytes):
    """(off uint64[n], len uint32[n] = size+1, kind uint8[n]) for every block of an SST image."""
    import numpy as np

    L = _sst_lib()
    n = ctypes.c_size_t(0)
    rc = L.leveldb_sst_block_spans(image, len(image), None, None, None, 0, ctypes.byref(n))
    if rc not in (0, SST_ECAPACITY):
        _raise(rc, L.leveldb_sst_last_error().decode())
    off = np.empty(n.value, dtype=np.uint64)
    ln = np.empty(n.value, dtype=np.uint32)
    kind = np.empty(n.value, dtype=np.uint8)
    rc = L.leveldb_sst_block_spans(image, len(image), off.ctypes.data, ln.ctypes.data, kind.ctypes.data, n.value,
                                   ctypes.byref(n))
    if rc != 0:
        _raise(rc, L.leveldb_sst_last_error().decode())
    return off, ln, kind


@dataclass
class BlockStatus:
    table: int
    kind: str
    offset: int
    size: int
    status: str


@dataclass
class VerifyResult:
    blocks: List[BlockStatus]
    table_errors: List[str]  # per table: "" or the layout Status text (Corruption / Not implemented)

    @property
    def ok(self) -> bool:
        return not any(self.table_errors) and all(b.status == OK for b in self.blocks)

    def bad_blocks(self) -> List[BlockStatus]:
        return [b for b in self.blocks if b.status != OK]


def verify_tables(images: Sequence[bytes], device=None, stream=None, check_bounds: bool = True) -> VerifyResult:
    """Verify every block of every SST image with one device batch.

    The images are packed back to back into one device buffer (as a compaction
    would stage its input files), spans are collected per image, and one
    leveldb_crc32c_batch with a mismatch vector covers them all.

    check_bounds: the spans (each with its 4-byte trailer) are checked against
    their image on the host, where they already are -- no device reduction or
    extra sync; the parser (leveldb_sst_block_spans) already rejects handles
    past the file, so False only skips this second look."""
    import numpy as np
    import torch

    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    offs, lens, kinds, tabs, errors, bases = [], [], [], [], [], []
    base = 0
    for t, img in enumerate(images):
        bases.append(base)
        try:
            o, ln, k = block_spans(img)
            errors.append("")
        except SstError as e:
            o, ln, k = (np.empty(0, np.uint64), np.empty(0, np.uint32), np.empty(0, np.uint8))
            errors.append(str(e))
        offs.append(o + np.uint64(base))
        lens.append(ln)
        kinds.append(k)
        if check_bounds and len(o) and int((o + ln.astype(np.uint64) + np.uint64(4)).max()) > len(img):
            raise ValueError(f"image {t}: a block span reaches past the file ({len(img)} bytes)")
        tabs.append(np.full(len(o), t, dtype=np.int64))
        base += (len(img) + 15) & ~15
    blob = np.zeros(base, dtype=np.uint8)
    for img, b in zip(images, bases):
        blob[b:b + len(img)] = np.frombuffer(img, dtype=np.uint8)
    off = np.concatenate(offs) if offs else np.empty(0, np.uint64)
    ln = np.concatenate(lens) if lens else np.empty(0, np.uint32)
    kind = np.concatenate(kinds) if kinds else np.empty(0, np.uint8)
    tab = np.concatenate(tabs) if tabs else np.empty(0, np.int64)
    blocks: List[BlockStatus] = []
    if len(off):
        # copies, batch and readback all on one stream (torch's current one
        # unless the caller names another), so each waits for the one before
        with torch.cuda.stream(stream) if stream is not None else nullcontext():
            d_buf = torch.from_numpy(blob).to(dev, non_blocking=True)
            d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
            d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
            _, mm = crc32c.batch(d_buf, d_off, d_len, verify=True, check_bounds=False)  # checked above
            bad = mm.cpu().numpy()
        for i in range(len(off)):
            t = int(tab[i])
            blocks.append(BlockStatus(t, KIND_NAMES[int(kind[i])], int(off[i]) - bases[t], int(ln[i]) - 1,
                                      MISMATCH if bad[i] else OK))
    return VerifyResult(blocks, errors)


def seal_blocks(buf, off, size, *, stream=None, check_bounds: bool = True):
    """Write `type || LE32(Mask(crc32c(contents || type)))` trailers in place.

    buf: device uint8 tensor holding blocks at off[i] (int64) with size[i]
    (int32) content bytes, the type byte already at off[i]+size[i]; the 4
    bytes after it are overwritten.  Returns the masked CRCs (int32).
    check_bounds as for crc32c.batch (True blocks the host on a device
    reduction; pass False for descriptors already checked)."""
    import torch

    with torch.cuda.stream(stream) if stream is not None else nullcontext():
        lens = size + 1
        out, _ = crc32c.batch(buf, off, lens, mask=True, trailer=True, check_bounds=check_bounds)
    return out
