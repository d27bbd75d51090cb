#!/usr/bin/env python3
"""Per-call cost of one SST-file-sized batch (16 811 data blocks of 3988 B at
stride 3992 + one 486 977-B index span, 67 MB), the granularity PrismDB seals
(TableBuilder::Finish) and verifies (a compaction input) at: device-resident,
one stream.

  back_to_back_us   100 calls enqueued without waiting, HIP events around
                    all of them, / 100 (what a compaction thread issuing file
                    after file sees)
  synced_us         median of 200 calls each waited for (includes the host
                    launch latency)

for the one-launch path (the default for <= 2^17 spans) and, pinned by the
test hook, the planner path; seal (MASK | WRITE_TRAILER), verify and plain,
seal / verify with PRISMDB_CRC32C_UNORDERED alternating between two
files (every other launch may overlap its predecessor), and seal / verify
rotating over eight distinct files (540 MB: not served from the MALL).
Prints one JSON object."""
import ctypes
import json
import os
import statistics
import sys

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")  # the library's prismdb_* setters act only with this
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from prismdb_amd import crc32c
    from prismdb_amd._lib import lib

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    nd = 16811
    size = nd * 3992 + 486977 + 64
    buf = torch.empty(size, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00F1)
    buf2 = buf.clone()  # a second file: unordered calls alternate between the two
    # eight distinct files (540 MB, over the 256 MB MALL): a compaction's
    # files are new data, while back-to-back calls on one file are partly
    # served from the MALL (profiles/r03ad_pmc_per_span.json)
    files = [torch.empty_like(buf) for _ in range(8)]
    for i, f in enumerate(files):
        crc32c.fill_synthetic(f, 0x5EED0100 + i)
    rot = [0]

    def next_file():
        rot[0] = (rot[0] + 1) % len(files)
        return files[rot[0]]
    off = np.concatenate([np.arange(nd, dtype=np.int64) * 3992, [nd * 3992]])
    lens = np.array([3988] * nd + [486977], dtype=np.int32)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    out = torch.empty(nd + 1, dtype=torch.int32, device=dev)
    mm = torch.empty(nd + 1, dtype=torch.uint8, device=dev)
    mm2 = torch.empty(nd + 1, dtype=torch.uint8, device=dev)
    crc32c.batch(buf, d_off, d_len, mask=True, trailer=True)  # seal once: verify then passes
    crc32c.batch(buf2, d_off, d_len, mask=True, trailer=True)
    flip = [0]

    def other():  # the file the previous unordered call did not touch
        flip[0] ^= 1
        return buf2 if flip[0] else buf
    s = torch.cuda.current_stream()

    def synced(fn, reps=200):
        for _ in range(10):
            fn()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return round(statistics.median(ts), 2)

    def b2b(fn, calls=100, reps=5):
        for _ in range(10):
            fn()
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(calls):
                fn()
            e1.record(s)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / calls
            best = us if best is None else min(best, us)
        return round(best, 2)

    modes = {
        "seal": lambda: crc32c.batch(buf, d_off, d_len, mask=True, trailer=True, out=out, check_bounds=False),
        "verify": lambda: crc32c.batch(buf, d_off, d_len, verify=True, out=out, mismatch=mm, check_bounds=False),
        "plain": lambda: crc32c.batch(buf, d_off, d_len, out=out, check_bounds=False),
        "data_only": lambda: crc32c.batch(buf, d_off[:nd], d_len[:nd], out=out[:nd], check_bounds=False),
        # seal / verify (the stored trailers do not match: results only) over eight distinct files in turn
        "seal_distinct": lambda: crc32c.batch(next_file(), d_off, d_len, mask=True, trailer=True, out=out,
                                              check_bounds=False),
        "verify_distinct": lambda: crc32c.batch(next_file(), d_off, d_len, verify=True, out=out, mismatch=mm2,
                                                check_bounds=False),
        # PRISMDB_CRC32C_UNORDERED: consecutive calls on two different files
        "seal_unordered": lambda: crc32c.batch(other(), d_off, d_len, mask=True, trailer=True, out=out,
                                               check_bounds=False, unordered=True),
        "verify_unordered": lambda: crc32c.batch(other(), d_off, d_len, verify=True, out=out, mismatch=mm,
                                                 check_bounds=False, unordered=True),
    }
    res = {"file": "16811 x 3988 B @ 3992 + 1 x 486977 B", "bytes": int(lens.astype(np.int64).sum())}
    native = lib()
    for route, dmax in (("one_launch", 1 << 17), ("planner", 0)):
        native.prismdb_crc32c_direct_max(dmax)
        for name, fn in modes.items():
            res[f"{route}_{name}_back_to_back_us"] = b2b(fn)
            res[f"{route}_{name}_synced_us"] = synced(fn)
    native.prismdb_crc32c_direct_max(1 << 17)
    assert int(mm.sum().item()) == 0
    # who folded the index span's tickets: per call, over 200 seal calls
    # (stats: adopted orphans, spans folded whole, worker claims, late claims)
    st = (ctypes.c_uint64 * 4)()
    modes["seal"]()
    torch.cuda.synchronize()
    assert native.prismdb_crc32c_direct_stats(st) == 0
    s0 = list(st)
    for _ in range(200):
        modes["seal"]()
    torch.cuda.synchronize()
    assert native.prismdb_crc32c_direct_stats(st) == 0
    res["one_launch_tickets_per_call"] = dict(zip(("adopted", "whole", "worker", "late"),
                                                  [round((b - a) / 200, 2) for a, b in zip(s0, st)]))
    res["fixed_data_blocks_back_to_back_us"] = b2b(lambda: crc32c.batch_fixed(buf, 3992, 3988, nd, out=out[:nd]))
    res["fixed_data_blocks_distinct_back_to_back_us"] = b2b(
        lambda: crc32c.batch_fixed(next_file(), 3992, 3988, nd, out=out[:nd]))
    res["ideal_us_at_8TBps"] = round(res["bytes"] / 8e12 * 1e6, 2)
    res["ideal_us_at_6.5TBps"] = round(res["bytes"] / 6.5e12 * 1e6, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
