#!/usr/bin/env python3
"""SST files per leveldb_crc32c_batch call: µs per file for k = 1..12 files
per call, sealing and verifying, through tools/variants.py builds: `base`
(one-launch limit 2^17 spans: 8+ files take two windows) and `direct196k`
(limit 196 608 spans: one launch while every wave's static run stays <= 64
spans, up to 11 files).

    python tools/variants.py build --only base direct196k
    python tools/files_per_call.py [lib ...]   # GPU box; one JSON object (default: base direct196k)

Each row: 143 distinct files (as bench's config5_partitions), calls of k
files back to back on one stream over them in turn, timed with events around
the whole sequence; µs per file."""
import ctypes
import json
import os
import sys

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ND, DATA, STRIDE, INDEX, NF = 16811, 3988, 3992, 486977, 143


def main():
    import numpy as np
    import torch

    from prismdb_amd import crc32c
    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    fb = (ND * STRIDE + INDEX + 4 + 255) & ~255
    off1 = np.concatenate([np.arange(ND, dtype=np.int64) * STRIDE, [ND * STRIDE]])
    len1 = np.concatenate([np.full(ND, DATA, dtype=np.int64), [INDEX]])
    off = (np.arange(NF, dtype=np.int64)[:, None] * fb + off1[None, :]).reshape(-1)
    lens = np.tile(len1, NF)
    buf = torch.empty(NF * fb, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0F11)
    buf[torch.from_numpy(off + lens).to(dev)] = 0
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    spf = ND + 1
    out = torch.empty(len(off), dtype=torch.int32, device=dev)
    mm = torch.empty(len(off), dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    crc32c.batch(buf, d_off, d_len, mask=True, trailer=True, out=out, check_bounds=False)  # sealed once
    torch.cuda.synchronize()
    res = {}
    for name in (sys.argv[1:] or ["base", "direct196k"]):
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "vlib", f"lib_{name}.so"), mode=os.RTLD_LOCAL)
        L.leveldb_crc32c_batch.restype = ctypes.c_int
        L.leveldb_crc32c_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                                                   ctypes.c_uint32, ctypes.c_void_p]
        row = {}
        for k in (1, 7, 8, 9, 10, 11, 12):
            calls = NF // k
            for verify in (False, True):
                def one(c):
                    a = c * k * spf
                    rc = L.leveldb_crc32c_batch(buf.data_ptr(), d_off.data_ptr() + 8 * a, d_len.data_ptr() + 4 * a, None,
                                                k * spf, out.data_ptr() + 4 * a,
                                                mm.data_ptr() + a if verify else None, 0 if verify else 3, sp)
                    assert rc == 0, rc
                for c in range(calls):
                    one(c)
                torch.cuda.synchronize()
                best = None
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for c in range(calls):
                        one(c)
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / (calls * k)
                    best = us if best is None else min(best, us)
                row[f"{k}_{'verify' if verify else 'seal'}"] = round(best, 2)
        res[name] = row
    assert int(mm.sum().item()) == 0
    print(json.dumps(res))


if __name__ == "__main__":
    main()
