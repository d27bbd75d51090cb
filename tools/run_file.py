#!/usr/bin/env python3
"""Driver for profiling the one-launch kernel at the per-file granularity:
`calls` calls over SST-shaped files (16 811 x 3988 B @ 3992 + the 486 977-B
index span each), back to back on one stream: seal (MASK | WRITE_TRAILER) by
default, or verify.  --files K lays out K distinct files and cycles through
them (K = 1: the same file every call, which the MALL then holds); --per-call
F passes F consecutive files per call.

    python tools/run_file.py [calls] [--files K] [--per-call F] [--verify]
    (tools/prof_file.sh runs it under rocprofv3)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("calls", type=int, nargs="?", default=20)
    ap.add_argument("--files", type=int, default=1)
    ap.add_argument("--per-call", type=int, default=1)
    ap.add_argument("--verify", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    nd = 16811
    fsz = nd * 3992 + 486977 + 4 + 3  # a file's spans, the index trailer, padding to a 4-B multiple
    k, f = args.files, args.per_call
    assert k % f == 0 and f * (nd + 1) <= 1 << 17
    buf = torch.empty(k * fsz + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00F1)
    one = np.concatenate([np.arange(nd, dtype=np.int64) * 3992, [nd * 3992]])
    off = torch.from_numpy((np.arange(k, dtype=np.int64)[:, None] * fsz + one[None, :]).reshape(-1)).to(dev)
    lens = torch.from_numpy(np.tile(np.array([3988] * nd + [486977], dtype=np.int32), k)).to(dev)
    out = torch.empty(k * (nd + 1), dtype=torch.int32, device=dev)
    mm = torch.empty(k * (nd + 1), dtype=torch.uint8, device=dev)
    # seal once so that verify finds its trailers
    for c in range(k // f):
        s = slice(c * f * (nd + 1), (c + 1) * f * (nd + 1))
        crc32c.batch(buf, off[s], lens[s], mask=True, trailer=True, out=out[s], check_bounds=False)
    torch.cuda.synchronize()
    for i in range(args.calls):
        c = i % (k // f)
        s = slice(c * f * (nd + 1), (c + 1) * f * (nd + 1))
        if args.verify:
            crc32c.batch(buf, off[s], lens[s], mask=True, verify=True, out=out[s], mismatch=mm[s], check_bounds=False)
        else:
            crc32c.batch(buf, off[s], lens[s], mask=True, trailer=True, out=out[s], check_bounds=False)
    torch.cuda.synchronize()
    if args.verify:
        assert int(mm.sum()) == 0
    print(f"{args.calls} calls of {f} file(s) over {k} done ({'verify' if args.verify else 'seal'})")


if __name__ == "__main__":
    main()
