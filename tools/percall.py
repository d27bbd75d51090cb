#!/usr/bin/env python3
"""Per-call latency of one SST-file-sized batch (16 811 data blocks of 3988 B at
stride 3992 + one 486 977-B index span), the granularity a compaction verifies
at: device-resident, HIP events around each call, median of many calls.
Prints one JSON object."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    nd = 16811
    size = nd * 3992 + 486977 + 64
    buf = torch.empty(size, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00F1)
    res = {}

    def timed(fn, reps=200):
        for _ in range(10):
            fn()
        ts = []
        s = torch.cuda.current_stream()
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return round(statistics.median(ts), 1)

    off = np.arange(nd, dtype=np.int64) * 3992
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.full((nd,), 3988, dtype=torch.int32, device=dev)
    out = torch.empty(nd + 1, dtype=torch.int32, device=dev)
    res["data_blocks_desc_us"] = timed(lambda: crc32c.batch(buf, d_off, d_len, out=out[:nd], check_bounds=False))
    off2 = torch.from_numpy(np.concatenate([off, [nd * 3992]])).to(dev)
    len2 = torch.from_numpy(np.array([3988] * nd + [486977], dtype=np.int32)).to(dev)
    res["sst_file_desc_us"] = timed(lambda: crc32c.batch(buf, off2, len2, out=out, check_bounds=False))
    res["data_blocks_fixed_us"] = timed(lambda: crc32c.batch_fixed(buf, 3992, 3988, nd, out=out[:nd]))
    bytes_ = nd * 3988
    res["data_bytes"] = bytes_
    res["ideal_us_at_6.5TBps"] = round(bytes_ / 6.5e12 * 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
