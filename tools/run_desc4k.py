#!/usr/bin/env python3
"""Workload driver for profiling the descriptor (span) kernel: 16 Mi x 4 KiB spans."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    n = 1 << 24
    buf = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    off = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        crc32c.batch(buf, off, lens, out=out, check_bounds=False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
