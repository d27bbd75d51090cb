#!/usr/bin/env python3
"""Host-resident rate of leveldb_crc32c_batch_host against the chunk size
(tuning hook prismdb_pipeline_chunk_bytes): 2 GiB of 4 KiB blocks from a
pinned and from a pageable source, next to the plain pinned H2D copy of the
same bytes (bench.py --e2e's legs, one process, chunk sizes interleaved per
rep; best of reps).  Every result is checked against the device batch.

    python tools/pipe_chunks.py [--mib 16 32 48 64] [--reps 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")  # the library's prismdb_* setters act only with this
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, nargs="*", default=[16, 32, 48, 64])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    from prismdb_amd import crc32c
    from prismdb_amd._lib import lib

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    nblk, blk = 1 << 19, 4096
    tmp = torch.empty(nblk * blk, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(tmp, 0x5EED0007)
    ref, _ = crc32c.batch_fixed(tmp, blk, blk, nblk)
    ref = ref.cpu().numpy().view(np.uint32)
    pinned = tmp.cpu().pin_memory()
    pageable = pinned.numpy().copy()
    del tmp
    off = np.arange(nblk, dtype=np.uint64) * blk
    lens = np.full(nblk, blk, dtype=np.uint32)
    out = np.empty(nblk, dtype=np.uint32)
    f = lib().leveldb_crc32c_batch_host
    hook = lib().prismdb_pipeline_chunk_bytes
    u64p, u32p = ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)

    def run(src_ptr):
        t0 = time.perf_counter()
        rc = f(ctypes.c_void_p(src_ptr), off.ctypes.data_as(u64p), lens.ctypes.data_as(u32p), None, nblk,
               out.ctypes.data_as(u32p), None, 0)
        el = time.perf_counter() - t0
        assert rc == 0, rc
        assert np.array_equal(out, ref)
        return nblk * blk / el / GIB

    res = {"bytes": nblk * blk, "reps": args.reps, "stat": "best of reps", "unit": "GiB/s", "rows": {}}
    prev = hook(0)
    try:
        for _ in range(args.reps):
            for mib in args.mib:
                hook(mib << 20)
                for name, ptr in (("pinned", pinned.data_ptr()), ("pageable", pageable.ctypes.data)):
                    key = f"{mib}MiB_{name}"
                    res["rows"][key] = max(res["rows"].get(key, 0.0), round(run(ptr), 2))
            d = torch.empty(nblk * blk, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d.copy_(pinned, non_blocking=True)
            torch.cuda.synchronize()
            res["rows"]["h2d_copy_only"] = max(res["rows"].get("h2d_copy_only", 0.0),
                                               round(nblk * blk / (time.perf_counter() - t0) / GIB, 2))
            del d
    finally:
        hook(prev)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
