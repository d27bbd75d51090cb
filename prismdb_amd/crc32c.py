"""Python face of leveldb::crc32c and of the MI355X batch engine.

Per-call surface (same names/meaning as util/crc32c.h:17-38):
    Extend(init_crc, data) -> int     crc32c(A || data) given init_crc = crc32c(A)
    Value(data) -> int                crc32c(data)
    Mask(crc) / Unmask(masked)        storage masking (rotate right 15 + kMaskDelta)
These run on the host (a GPU launch per 4 KiB call would lose), through the
native library's leveldb::crc32c::Extend.

Batch surface (device-resident spans, one call = one batch of SST blocks):
    batch_fixed(buf, stride, length, nblocks, ...)   block i = buf[i*stride : i*stride+length]
    batch(buf, off, lens, init=None, ...)            span i  = buf[off[i] : off[i]+lens[i]]
    batch_multi([(buf, off, lens), ...], ...)        one partition per device, results gathered
                                                     to the first partition's device (RCCL)
buf/off/lens/init/out are torch tensors on the current HIP device; calls are
enqueued on torch's current stream.  mask=True applies Mask() to each result
(TableBuilder::WriteRawBlock, table/table_builder.cc:194-196); verify=True also
returns a per-span uint8 mismatch flag comparing Value(span) with
Unmask(LE32(trailer at span end)) (ReadBlock, table/format.cc:91-102 with
span = contents||type).  A mismatch is data: callers turn it into
Status::Corruption("block checksum mismatch"), see prismdb_amd.sst.
"""
from __future__ import annotations

import ctypes
from contextlib import nullcontext as _nullcontext
from typing import Optional, Tuple

from ._lib import check, lib

kMaskDelta = 0xA282EAD8
FLAG_MASK = 0x1
FLAG_WRITE_TRAILER = 0x2
FLAG_LOG_HEADER = 0x4
FLAG_UNORDERED = 0x8


def _bytes(data) -> bytes:
    if isinstance(data, str):
        return data.encode("latin-1")
    return bytes(data)


def Extend(init_crc: int, data) -> int:
    b = _bytes(data)
    return lib().leveldb_crc32c_extend(init_crc & 0xFFFFFFFF, b, len(b))


def Value(data) -> int:
    b = _bytes(data)
    return lib().leveldb_crc32c_value(b, len(b))


def Mask(crc: int) -> int:
    return lib().leveldb_crc32c_mask(crc & 0xFFFFFFFF)


def Unmask(masked_crc: int) -> int:
    return lib().leveldb_crc32c_unmask(masked_crc & 0xFFFFFFFF)


def Combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """crc32c(A || B) from crc32c(A), crc32c(B) and len(B)."""
    return lib().leveldb_crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)


def accelerated() -> bool:
    """True if the host Extend uses the CPU's CRC32 instruction (KAT-gated)."""
    return bool(lib().leveldb_crc32c_accelerated())


# ---------------------------------------------------------------- device batch


def _torch():
    import torch

    return torch


def _stream_ptr(stream) -> int:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def device_init(device: int = 0) -> None:
    check(lib().leveldb_crc32c_device_init(device), "leveldb_crc32c_device_init")


def _require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise ValueError("batch inputs must be device tensors (the engine has no CPU path)")


def batch_fixed(buf, stride: int, length: int, nblocks: int, init: int = 0, *, mask: bool = False,
                verify: bool = False, out=None, mismatch=None, stream=None) -> Tuple[object, Optional[object]]:
    """CRC32C of nblocks fixed-stride blocks of a device buffer.

    Returns (out uint32-as-int32 tensor [nblocks], mismatch uint8 [nblocks] or None).
    """
    torch = _torch()
    _require_device(buf)
    if nblocks and (nblocks - 1) * stride + length + (4 if verify else 0) > buf.numel() * buf.element_size():
        raise ValueError("blocks extend past the end of buf")
    if out is None:
        out = torch.empty(nblocks, dtype=torch.int32, device=buf.device)
    if verify and mismatch is None:
        mismatch = torch.empty(nblocks, dtype=torch.uint8, device=buf.device)
    rc = lib().leveldb_crc32c_batch_fixed(
        buf.data_ptr(), stride, length, nblocks, init & 0xFFFFFFFF, out.data_ptr(),
        mismatch.data_ptr() if verify else None, FLAG_MASK if mask else 0, _stream_ptr(stream))
    check(rc, "leveldb_crc32c_batch_fixed")
    return out, (mismatch if verify else None)


def _span_reach(log_header: bool, verify: bool, trailer: bool) -> Tuple[int, int]:
    """(bytes read or written before a span, bytes after it): the stored log
    header (6 B before, LOG_HEADER with verify or trailer) or the 4-byte block
    trailer after it (verify or trailer without LOG_HEADER)."""
    touches = verify or trailer
    return (6 if touches and log_header else 0), (4 if touches and not log_header else 0)


def batch(buf, off, lens, init=None, *, mask: bool = False, verify: bool = False, out=None,
          mismatch=None, stream=None, trailer: bool = False, log_header: bool = False,
          check_bounds: bool = True, unordered: bool = False) -> Tuple[object, Optional[object]]:
    """CRC32C of arbitrary spans buf[off[i] : off[i]+lens[i]] (int64 off, int32 lens, int32 init).

    trailer=True also stores each (masked, with mask=True) result as 4 LE bytes
    right after its span (TableBuilder::WriteRawBlock).

    check_bounds: every span, with its stored trailer or log header, must lie
    inside buf (ValueError otherwise; a bad descriptor would be a device
    fault).  The check is one device reduction and a host sync, so with the
    default the call blocks the host even when `stream` is given; callers
    that reuse descriptors they have already checked pass False and stay
    asynchronous.

    unordered: PRISMDB_CRC32C_UNORDERED, accepted and ignored (every batch
    runs in stream order; see include/prismdb_crc32c.h)."""
    if trailer and verify:
        raise ValueError("trailer and verify are exclusive")
    torch = _torch()
    _require_device(buf, off, lens, init)
    n = off.numel()
    if lens.numel() != n or (init is not None and init.numel() != n):
        raise ValueError("off, lens and init must have the same length")
    if off.dtype != torch.int64 or lens.dtype != torch.int32 or (init is not None and init.dtype != torch.int32):
        raise TypeError("off must be int64, lens/init int32 (uint32 bit patterns)")
    off, lens = off.contiguous(), lens.contiguous()
    if check_bounds and n:
        lead, tail = _span_reach(log_header, verify, trailer)
        with torch.cuda.stream(stream) if stream is not None else _nullcontext():
            end = off + (lens.to(torch.int64) & 0xFFFFFFFF)
            lo, omax, hi = torch.stack([off.min(), off.max(), end.max()]).tolist()
        # 0 <= off <= size for every span first: then no off + len wraps
        size = buf.numel() * buf.element_size()
        if lo < lead or omax > size or hi + tail > size:
            raise ValueError(f"spans reach [{lo - lead}, {hi + tail}) outside buf "
                             f"({buf.numel() * buf.element_size()} bytes)")
    init = init.contiguous() if init is not None else None
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=buf.device)
    if verify and mismatch is None:
        mismatch = torch.empty(n, dtype=torch.uint8, device=buf.device)
    rc = lib().leveldb_crc32c_batch(
        buf.data_ptr(), off.data_ptr(), lens.data_ptr(), init.data_ptr() if init is not None else None, n,
        out.data_ptr(), mismatch.data_ptr() if verify else None,
        (FLAG_MASK if mask else 0) | (FLAG_WRITE_TRAILER if trailer else 0) | (FLAG_LOG_HEADER if log_header else 0)
        | (FLAG_UNORDERED if unordered else 0),
        _stream_ptr(stream))
    check(rc, "leveldb_crc32c_batch")
    return out, (mismatch if verify else None)


def batch_multi(parts, *, mask: bool = False, verify: bool = False, trailer: bool = False,
                log_header: bool = False, out=None, mismatch=None, streams=None, check_bounds: bool = True):
    """Partitions on several devices from one process
    (leveldb_crc32c_batch_multi): parts[p] = (buf, off, lens[, init]) device
    tensors on one device each (distinct devices; parts[0]'s is the root).
    Every device checksums its partition, and an RCCL gather brings the
    results to the root device, partition after partition.

    Returns (out int32 tensor [sum n] on the root device, mismatch uint8 or
    None).  streams: None (each device's current stream) or one torch stream
    per part."""
    torch = _torch()
    if trailer and verify:
        raise ValueError("trailer and verify are exclusive")
    if not parts:
        raise ValueError("batch_multi needs at least one partition")
    ndev = len(parts)
    devs, bases, offs, lns, inits, ns = [], [], [], [], [], []
    for p, part in enumerate(parts):
        buf, off, lens = part[0], part[1], part[2]
        init = part[3] if len(part) > 3 else None
        _require_device(buf, off, lens, init)
        d = buf.device.index
        for t in (off, lens, init):
            if t is not None and t.device != buf.device:
                raise ValueError(f"partition {p}: its tensors must be on one device")
        if off.dtype != torch.int64 or lens.dtype != torch.int32 or (init is not None and init.dtype != torch.int32):
            raise TypeError("off must be int64, lens/init int32 (uint32 bit patterns)")
        n = off.numel()
        if lens.numel() != n or (init is not None and init.numel() != n):
            raise ValueError(f"partition {p}: off, lens and init must have the same length")
        off, lens = off.contiguous(), lens.contiguous()
        init = init.contiguous() if init is not None else None
        if check_bounds and n:
            lead, tail = _span_reach(log_header, verify, trailer)
            with torch.cuda.device(d):
                end = off + (lens.to(torch.int64) & 0xFFFFFFFF)
                lo, omax, hi = torch.stack([off.min(), off.max(), end.max()]).tolist()
            size = buf.numel() * buf.element_size()
            if lo < lead or omax > size or hi + tail > size:
                raise ValueError(f"partition {p}: spans reach [{lo - lead}, {hi + tail}) outside its buffer")
        devs.append(d)
        bases.append(buf.data_ptr())
        offs.append(off)
        lns.append(lens)
        inits.append(init)
        ns.append(n)
    if len(set(devs)) != ndev:
        raise ValueError("batch_multi: one partition per device")
    total = sum(ns)
    root = torch.device("cuda", devs[0])
    if out is None:
        out = torch.empty(total, dtype=torch.int32, device=root)
    if verify and mismatch is None:
        mismatch = torch.empty(total, dtype=torch.uint8, device=root)
    # the C side writes n[0] + ... + n[ndev-1] entries at out / mismatch on the root device
    for name, t, dt in (("out", out, torch.int32), ("mismatch", mismatch if verify else None, torch.uint8)):
        if t is None:
            continue
        if t.dtype != dt or t.device != root or not t.is_contiguous() or t.numel() < total:
            raise ValueError(f"batch_multi: {name} must be a contiguous {dt} tensor of >= {total} entries "
                             f"on {root} (got {t.dtype}, {t.numel()} on {t.device})")
    P = ctypes.c_void_p * ndev
    c_dev = (ctypes.c_int * ndev)(*devs)
    c_base = P(*bases)
    c_off = P(*[t.data_ptr() for t in offs])
    c_len = P(*[t.data_ptr() for t in lns])
    c_init = P(*[t.data_ptr() if t is not None else None for t in inits])
    c_n = (ctypes.c_size_t * ndev)(*ns)
    if streams is None:
        streams = [torch.cuda.current_stream(d) for d in devs]
    c_st = P(*[int(s.cuda_stream) for s in streams])
    flags = (FLAG_MASK if mask else 0) | (FLAG_WRITE_TRAILER if trailer else 0) | (FLAG_LOG_HEADER if log_header else 0)
    keep = (offs, lns, inits)  # alive until the call has enqueued its work  # noqa: F841
    rc = lib().leveldb_crc32c_batch_multi(ndev, c_dev, c_base, c_off, c_len,
                                          c_init if any(t is not None for t in inits) else None, c_n,
                                          out.data_ptr(), mismatch.data_ptr() if verify else None, flags, c_st)
    check(rc, "leveldb_crc32c_batch_multi")
    return out, (mismatch if verify else None)


def multi_timing(devices):
    """Phases of the last batch_multi call on this device list (diagnostics,
    HIP events on the clique's streams): {"batch_ms": [per device],
    "gather_ms": [per device], "init_ms": ncclCommInitAll's wall time}, or
    None if there was no such call."""
    ndev = len(devices)
    c_dev = (ctypes.c_int * ndev)(*devices)
    b, g = (ctypes.c_float * ndev)(), (ctypes.c_float * ndev)()
    init = ctypes.c_double(0)
    rc = lib().prismdb_crc32c_multi_timing(ndev, c_dev, b, g, ctypes.byref(init))
    if rc != 0:
        return None
    return {"batch_ms": [round(x, 3) for x in b], "gather_ms": [round(x, 3) for x in g],
            "init_ms": round(init.value, 1)}


def multi_host_timing(devices):
    """Host wall times of the last batch_multi call on this device list
    (diagnostics): {"start_us": [per device: call entry to the start of that
    partition's enqueue], "enqueue_us": [per device: the enqueue itself --
    hand-off, scratch, batch launches], "call_us": the whole call}, or None."""
    ndev = len(devices)
    c_dev = (ctypes.c_int * ndev)(*devices)
    st, en = (ctypes.c_double * ndev)(), (ctypes.c_double * ndev)()
    call = ctypes.c_double(0)
    if lib().prismdb_crc32c_multi_host_timing(ndev, c_dev, st, en, ctypes.byref(call)) != 0:
        return None
    return {"start_us": [round(x, 1) for x in st], "enqueue_us": [round(x, 1) for x in en],
            "call_us": round(call.value, 1)}


def batch_host(base, off, lens, init=None, *, mask: bool = False, verify: bool = False, log_header: bool = False,
               trailer: bool = False):
    """Host-resident batch: numpy (or pinned torch CPU tensor) buffer and
    descriptors in host memory; streamed through the device by the engine.
    trailer=True stores each (masked, with mask=True) result into `base` as
    the span's trailer (4 LE bytes after it; with log_header, the record
    header's crc 6 bytes before it), as TableBuilder::WriteRawBlock does.
    Returns (crc uint32[n], mismatch uint8[n] or None) as numpy arrays."""
    import numpy as np

    if trailer and verify:
        raise ValueError("trailer and verify are exclusive")

    n = len(off)
    off = np.asarray(off)
    if n and off.dtype.kind == "i" and int(off.min()) < 0:  # before the cast: -1 would wrap to 2^64 - 1
        raise ValueError("negative span offset")
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    ini = np.ascontiguousarray(init, dtype=np.uint32) if init is not None else None
    if len(lens) != n or (ini is not None and len(ini) != n):
        raise ValueError("off, lens and init must have the same length")
    # nbytes and the base pointer below assume one contiguous buffer; sealing
    # also writes into it (the C side refuses a read-only mapping, but a
    # read-only numpy view of a bytes object is writable memory it must not touch)
    if hasattr(base, "data_ptr"):
        if base.is_cuda or not base.is_contiguous():
            raise ValueError("batch_host: base must be a contiguous host tensor")
    else:
        if not base.flags.c_contiguous:
            raise ValueError("batch_host: base must be a C-contiguous array")
        if trailer and not base.flags.writeable:
            raise ValueError("batch_host: trailer=True writes into base, which is read-only")
    nbytes = base.numel() * base.element_size() if hasattr(base, "data_ptr") else base.nbytes
    if n:
        lead, tail = _span_reach(log_header, verify, trailer)
        lo, omax = int(off.min()), int(off.max())
        # 0 <= off <= nbytes for every span first: then no off + len wraps
        hi = int((off + lens.astype(np.uint64)).max()) if omax <= nbytes else omax
        if lo < lead or omax > nbytes or hi + tail > nbytes:
            raise ValueError(f"spans reach [{lo - lead}, {hi + tail}) outside the host buffer ({nbytes} bytes)")
    out = np.empty(n, dtype=np.uint32)
    mm = np.empty(n, dtype=np.uint8) if verify else None
    ptr = base.data_ptr() if hasattr(base, "data_ptr") else base.ctypes.data
    rc = lib().leveldb_crc32c_batch_host(ptr, off.ctypes.data, lens.ctypes.data,
                                         ini.ctypes.data if ini is not None else None, n, out.ctypes.data,
                                         mm.ctypes.data if verify else None,
                                         (FLAG_MASK if mask else 0) | (FLAG_LOG_HEADER if log_header else 0)
                                         | (FLAG_WRITE_TRAILER if trailer else 0))
    check(rc, "leveldb_crc32c_batch_host")
    return out, mm


def fill_synthetic(buf, seed: int, byte_offset: int = 0, stream=None) -> None:
    """Fill a device buffer with the splitmix64 stream (see include/prismdb_synth.h)."""
    _require_device(buf)
    rc = lib().prismdb_fill_synthetic(buf.data_ptr(), buf.numel() * buf.element_size(), seed & (2**64 - 1),
                                      byte_offset, _stream_ptr(stream))
    if rc != 0:
        raise RuntimeError(f"prismdb_fill_synthetic failed ({rc})")


def as_u32(t):
    """View an int32 result tensor as Python ints in [0, 2^32)."""
    return [int(x) & 0xFFFFFFFF for x in t.tolist()]
