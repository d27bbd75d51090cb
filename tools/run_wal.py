#!/usr/bin/env python3
"""Workload driver for profiling the log-record span kernel: WAL verify over
4 GiB of ~1 KB log records (the bench_configs wal_verify shape)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import numpy as np
    import torch

    from bench_configs import build_log
    from prismdb_amd import crc32c, log

    dev = torch.device("cuda", 0)
    fb, nf = 4 << 20, 1024
    rng = np.random.default_rng(0x5EED0003)
    img = build_log(rng, fb)
    hoff, hlen = log.scan(img)
    buf = torch.empty(nf * fb, dtype=torch.uint8, device=dev)
    buf.view(nf, fb).copy_(torch.from_numpy(img).to(dev))
    off = torch.from_numpy(((np.arange(nf, dtype=np.int64)[:, None] * fb + hoff.astype(np.int64)[None, :]) + 6)
                           .reshape(-1)).to(dev)
    ln = torch.from_numpy(np.tile(hlen.astype(np.int32) + 1, nf)).to(dev)
    crc32c.batch(buf, off, ln, mask=True, trailer=True, log_header=True)  # seal the headers
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        crc32c.batch(buf, off, ln, verify=True, log_header=True, check_bounds=False)
    torch.cuda.synchronize()
    print("records", off.numel())


if __name__ == "__main__":
    main()
