#!/usr/bin/env python3
"""Workload driver for profiling bulk SST descriptor batches (planner path,
pair-run kernel): 16 Mi SST spans -- 3988-B contents||type at stride 3992,
one 486 977-B index span per 16 811 -- plain, sealed (MASK | WRITE_TRAILER)
or verified, K calls.

    python tools/run_sst.py [plain|seal|verify] [K]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from prismdb_amd import crc32c

    mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    nd, stride, dl, il = 16811, 3992, 3988, 486977
    files = (1 << 24) // (nd + 1)
    fb = nd * stride + il + 4
    off1 = np.concatenate([np.arange(nd, dtype=np.int64) * stride, [nd * stride]])
    len1 = np.concatenate([np.full(nd, dl, dtype=np.int64), [il]])
    off = (np.arange(files, dtype=np.int64)[:, None] * fb + off1[None, :]).reshape(-1)
    lens = np.tile(len1, files)
    buf = torch.empty(files * fb + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    out = torch.empty(len(off), dtype=torch.int32, device=dev)
    if mode == "verify":
        crc32c.batch(buf, d_off, d_len, out=out, mask=True, trailer=True)
    for _ in range(k):
        crc32c.batch(buf, d_off, d_len, out=out, mask=mode == "seal", trailer=mode == "seal",
                     verify=mode == "verify", check_bounds=False)
    torch.cuda.synchronize()
    print(f"{mode}: {len(off)} spans x {k} calls")


if __name__ == "__main__":
    main()
