#!/usr/bin/env python3
"""Host time of one leveldb_crc32c_batch call (the enqueue, not the device
work) for each library built by tools/variants.py, on a config-5 partition
(2 404 116 SST spans, planner path) and on one SST file (one-launch path).

    python tools/host_enqueue.py --only base r05     # GPU box; one JSON object

Per library and shape: `calls` calls back to back on one stream, each timed
with time.perf_counter_ns around the C call (ctypes overhead included, the
same for every library), then a synchronize; median and p90 in us."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "tools", "vlib")
ND, DATA, STRIDE, INDEX = 16811, 3988, 3992, 486977


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="+", default=["base"])
    ap.add_argument("--calls", type=int, default=30)
    args = ap.parse_args()
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    nfiles = 143
    fbytes = (ND * STRIDE + INDEX + 4 + 255) & ~255
    off1 = np.concatenate([np.arange(ND, dtype=np.int64) * STRIDE, [ND * STRIDE]])
    len1 = np.concatenate([np.full(ND, DATA, dtype=np.int64), [INDEX]])
    off = (np.arange(nfiles, dtype=np.int64)[:, None] * fbytes + off1[None, :]).reshape(-1)
    lens = np.tile(len1, nfiles)
    buf = torch.empty(nfiles * fbytes, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00E1)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    out = torch.empty(len(off), dtype=torch.int32, device=dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for name in args.only:
        L = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"), mode=os.RTLD_LOCAL)
        f = L.leveldb_crc32c_batch
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.c_void_p]
        res[name] = {}
        for shape, n in (("config5_partition_seal", len(off)), ("one_file_seal", ND + 1)):
            for _ in range(3):
                assert f(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, n, out.data_ptr(), None, 3, sp) == 0
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.calls):
                t0 = time.perf_counter_ns()
                rc = f(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, n, out.data_ptr(), None, 3, sp)
                ts.append((time.perf_counter_ns() - t0) / 1e3)
                assert rc == 0
            torch.cuda.synchronize()
            ts.sort()
            res[name][shape] = {"median_us": round(statistics.median(ts), 1), "p90_us": round(ts[int(0.9 * len(ts))], 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
