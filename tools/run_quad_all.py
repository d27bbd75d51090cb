#!/usr/bin/env python3
"""Profiling driver: 4 Mi x 4 KiB descriptor spans (16 GiB) with every
descriptor batch routed through the quad kernel (prismdb_crc32c_quad_mode(1)),
then the same batch on the default path; for rocprofv3 kernel traces."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from prismdb_amd import _lib, crc32c

    dev = torch.device("cuda", 0)
    n = 1 << 22
    buf = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    off = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    L = _lib.lib()
    L.prismdb_crc32c_quad_mode.argtypes = [ctypes.c_int]
    for mode in (1, 0):
        L.prismdb_crc32c_quad_mode(mode)
        for _ in range(3):
            crc32c.batch(buf, off, lens, out=out, check_bounds=False)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
