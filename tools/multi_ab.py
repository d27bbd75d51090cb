#!/usr/bin/env python3
"""What one leveldb_crc32c_batch_multi call costs over the same batch issued
with leveldb_crc32c_batch on the caller's stream (measurement support).

    python tools/variants.py build --only base multi_notime ...   # here
    python tools/multi_ab.py --only base multi_notime             # GPU box

One device (ndev = 1: no gather), config 5's per-device batch (2.4 M SST-
shaped spans sealed), each library's batch_multi and plain batch calls
interleaved, back to back on one stream; prints ms per call (median of reps
of `--calls` calls each).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "tools", "vlib")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="+", default=["base"])
    ap.add_argument("--spans", type=int, default=2404116)
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    n = args.spans
    buf = torch.empty(n * 3992 + 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0C55)
    off = torch.arange(n, dtype=torch.int64, device=dev) * 3992
    lens = torch.full((n,), 3988, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    vp = ctypes.c_void_p
    calls = {}
    for name in args.only:
        lib = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"), mode=os.RTLD_LOCAL)
        m = lib.leveldb_crc32c_batch_multi
        m.restype = ctypes.c_int
        m.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_uint32, vp]
        b = lib.leveldb_crc32c_batch
        b.restype = ctypes.c_int
        b.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_uint32, vp]
        devs = (ctypes.c_int * 1)(0)
        bases = (vp * 1)(buf.data_ptr())
        offs = (vp * 1)(off.data_ptr())
        lns = (vp * 1)(lens.data_ptr())
        ns = (ctypes.c_size_t * 1)(n)
        strs = (vp * 1)(stream.cuda_stream)
        calls[name + ":multi"] = (lambda m=m, devs=devs, bases=bases, offs=offs, lns=lns, ns=ns, strs=strs:
                                  m(1, devs, bases, offs, lns, None, ns, out.data_ptr(), None, 0x3, strs))
        calls[name + ":batch"] = (lambda b=b: b(buf.data_ptr(), off.data_ptr(), lens.data_ptr(), None, n,
                                                out.data_ptr(), None, 0x3, sp))

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.calls):
            assert fn() == 0
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / args.calls

    names = list(calls)
    for k in names:
        timed(calls[k])
    res = {k: [] for k in names}
    for rep in range(args.reps):
        for k in (names if rep % 2 == 0 else names[::-1]):
            res[k].append(timed(calls[k]))
    print(json.dumps({"spans": n, "calls_per_rep": args.calls, "reps": args.reps,
                      "ms_per_call_median": {k: round(statistics.median(v), 4) for k, v in res.items()}}))
    _ = np


if __name__ == "__main__":
    main()
