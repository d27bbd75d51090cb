#!/usr/bin/env python3
"""Per-call floor of the engine's launches: HIP-event time of back-to-back calls
on tiny and SST-file-sized batches (fixed and descriptor paths).  Prints JSON."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    buf = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00F2)
    stream = torch.cuda.current_stream()
    res = {}

    def timed(fn, calls=100):
        for _ in range(10):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(calls):
            fn()
        e1.record(stream)
        e1.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / calls, 2)

    for n in (1, 64, 4096, 16811):
        out = torch.empty(n, dtype=torch.int32, device=dev)
        res[f"fixed_n{n}_us"] = timed(lambda: crc32c.batch_fixed(buf, 3992, 3988, n, out=out))
        off = torch.arange(n, dtype=torch.int64, device=dev) * 3992
        ln = torch.full((n,), 3988, dtype=torch.int32, device=dev)
        res[f"desc_n{n}_us"] = timed(lambda: crc32c.batch(buf, off, ln, out=out, check_bounds=False))
    x = torch.empty(1 << 20, dtype=torch.int32, device=dev)
    res["torch_fill_1m_us"] = timed(lambda: x.fill_(1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
