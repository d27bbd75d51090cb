#!/usr/bin/env python3
"""Driver for profiling the one-launch kernel at the per-file granularity:
`calls` seal calls (MASK | WRITE_TRAILER) of one SST-shaped file (16 811 x
3988 B @ 3992 + the 486 977-B index span), back to back on one stream.

    python tools/run_file.py [calls]        (tools/prof_file.sh runs it under rocprofv3)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    nd = 16811
    buf = torch.empty(nd * 3992 + 486977 + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00F1)
    off = torch.from_numpy(np.concatenate([np.arange(nd, dtype=np.int64) * 3992, [nd * 3992]])).to(dev)
    lens = torch.from_numpy(np.array([3988] * nd + [486977], dtype=np.int32)).to(dev)
    out = torch.empty(nd + 1, dtype=torch.int32, device=dev)
    for _ in range(calls):
        crc32c.batch(buf, off, lens, mask=True, trailer=True, out=out, check_bounds=False)
    torch.cuda.synchronize()
    print(f"{calls} file calls done")


if __name__ == "__main__":
    main()
