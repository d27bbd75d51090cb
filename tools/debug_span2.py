#!/usr/bin/env python3
"""Debug helper: compare the descriptor (span) kernel with the fixed kernel on
growing batches of 4 KiB blocks and print where they differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    nmax = 1 << 24
    buf = torch.empty(nmax * 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    nwaves = 256 * 16
    for n in (1 << 16, 1 << 20, 1 << 24, 1 << 24):
        out, _ = crc32c.batch_fixed(buf, 4096, 4096, n)
        off = torch.arange(n, dtype=torch.int64, device=dev) * 4096
        lens = torch.full((n,), 4096, dtype=torch.int32, device=dev)
        for rep in range(4):
            out2, _ = crc32c.batch(buf, off, lens)
            bad = (out != out2).nonzero().flatten().cpu()
            line = f"n={n} rep={rep} mismatches={bad.numel()}"
            if bad.numel():
                b = bad[:12].tolist()
                dec = [(x % nwaves, (x // nwaves) % 2, (x // nwaves) // 2) for x in b]
                line += f" first={b} (wave,stream,q)={dec}"
                waves = torch.unique(bad % nwaves).numel()
                qs = bad // nwaves // 2
                line += f" distinct_waves={waves} q_min={int(qs.min())} q_max={int(qs.max())}"
            print(line, flush=True)
        # same spans in a shuffled order of descriptors
    del buf


if __name__ == "__main__":
    main()
