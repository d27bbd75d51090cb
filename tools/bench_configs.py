#!/usr/bin/env python3
"""Secondary workloads of BASELINE.json (the headline is bench.py).

    python tools/bench_configs.py [--reps 5]

Prints one JSON object with, per workload, the mean kernel-sequence time
(HIP events on the launch stream), payload GiB/s and the HBM roofline fraction
of the algorithmic bytes (fixed L+4; variable L+4+12; verify
L+4+1 per span):
  config3_mixed      spans of 1/4/16/64 KiB (uniform, seed 0x5EED0003) packed back to back, ~16 GiB
  *_windows          the same batch as windows of 2^17 spans of the one-launch kernel, back to back
                     (the default for > 2^18 spans is the planner path)
  config3_band       200 000 of those spans: the 2^17..2^18 band whose default is two windows;
                     *_planner the planner path pinned
  sst_fixed          3988-B spans (YCSB data block + type byte) at stride 3992, 16 Mi spans (~62.4 GiB)
  sst_desc           same spans through descriptors + one 486 977-B index span per 16 811 (split path)
  verify_4k          ReadBlock-verify of 16 Mi x (4092 + type... ) 4 KiB spans with stored trailers
  adversarial        random lengths 0..70 000 at random byte offsets (2 Mi spans over 16 GiB)
  wal_verify         log::Reader's record check over 4096 x 4 MiB log files of ~1 KB records
                     (PrismDB YCSB WriteBatch size), LOG_HEADER verify: L+4+1+12 per record
  wal_seal           log::Writer's header crc for the same records, written in place: L+4+12
"""
import argparse
import json
import os
import statistics
import sys

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")  # the library's prismdb_* setters act only with this
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", nargs="*", help="workloads to run (default: all); e.g. wal_seal wal_verify")
    args = ap.parse_args()

    def want(*names):
        return not args.only or any(n in args.only for n in names)
    import numpy as np
    import torch
    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()

    def timed(fn, reps, k=3):
        # k calls back to back per timing, as a caller streams them: the
        # Python wrapper's work for call i+1 overlaps call i on the device
        # (timed one at a time, the first call's host work sat inside the
        # events: ~0.1 ms, 3-4 % of a WAL or config-3 call)
        ts = []
        fn()
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(k):
                fn()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3 / k)
        return statistics.median(ts)

    res = {}
    from prismdb_amd._lib import lib as native

    def windows(fn):  # the same call as windows of the one-launch kernel (default: the planner path)
        def run():
            prev = native().prismdb_crc32c_windows(1)
            try:
                fn()
            finally:
                native().prismdb_crc32c_windows(prev)
        return run

    def report(name, t, payload, algo, n):
        res[name] = {"spans": n, "payload_GiB": round(payload / GIB, 2), "ms": round(t * 1e3, 3),
                     "GiB/s": round(payload / t / GIB, 1), "algo_GB/s": round(algo / t / 1e9, 1),
                     "roofline_frac": round(algo / t / 8e12, 4)}

    # one 64 GiB buffer serves every workload
    buf = torch.empty(64 << 30, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)

    # config 3: mixed sizes
    rng = np.random.default_rng(0x5EED0003)
    lens = rng.choice([1024, 4096, 16384, 65536], size=(16 << 30) // 21760).astype(np.int64)
    if want("config3_mixed"):
        off = np.concatenate([[0], np.cumsum(lens)[:-1]])
        d_off, d_len = torch.from_numpy(off).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev)
        out = torch.empty(len(lens), dtype=torch.int32, device=dev)
        fn = lambda: crc32c.batch(buf, d_off, d_len, out=out, check_bounds=False)  # noqa: E731
        report("config3_mixed", timed(fn, args.reps), lens.sum(), lens.sum() + 16 * len(lens), len(lens))
        ref = out.clone()
        report("config3_mixed_windows", timed(windows(fn), args.reps), lens.sum(), lens.sum() + 16 * len(lens),
               len(lens))
        res["config3_mixed_windows"]["agrees"] = bool(torch.equal(ref, out))
        del d_off, d_len, out
    if want("config3_band"):
        # 200 000 config-3 spans: inside 2^17 < n <= 2^18, where the default
        # route is two windows of the one-launch kernel; the planner path (and
        # the windows pinned) next to it
        m = 200_000
        bl = lens[:m]
        off = np.concatenate([[0], np.cumsum(bl)[:-1]])
        d_off, d_len = torch.from_numpy(off).to(dev), torch.from_numpy(bl.astype(np.int32)).to(dev)
        out = torch.empty(m, dtype=torch.int32, device=dev)
        fn = lambda: crc32c.batch(buf, d_off, d_len, out=out, check_bounds=False)  # noqa: E731
        report("config3_band", timed(fn, args.reps), bl.sum(), bl.sum() + 16 * m, m)
        ref = out.clone()

        def planner():
            prev = native().prismdb_crc32c_windows(0)
            try:
                fn()
            finally:
                native().prismdb_crc32c_windows(prev)
        report("config3_band_planner", timed(planner, args.reps), bl.sum(), bl.sum() + 16 * m, m)
        res["config3_band_planner"]["agrees"] = bool(torch.equal(ref, out))
        report("config3_band_windows", timed(windows(fn), args.reps), bl.sum(), bl.sum() + 16 * m, m)
        del d_off, d_len, out
    if want("config3_seal"):
        # the same span sizes sealed (MASK | WRITE_TRAILER): a 4-B trailer slot after each span
        off = np.concatenate([[0], np.cumsum(lens + 4)[:-1]])
        d_off, d_len = torch.from_numpy(off).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev)
        out = torch.empty(len(lens), dtype=torch.int32, device=dev)
        fn = lambda: crc32c.batch(buf, d_off, d_len, out=out, mask=True, trailer=True, check_bounds=False)  # noqa: E731
        report("config3_seal", timed(fn, args.reps), lens.sum(), lens.sum() + 20 * len(lens), len(lens))
        ref = out.clone()
        report("config3_seal_windows", timed(windows(fn), args.reps), lens.sum(), lens.sum() + 20 * len(lens),
               len(lens))
        res["config3_seal_windows"]["agrees"] = bool(torch.equal(ref, out))
        del d_off, d_len, out

    # SST-shaped, fixed stride
    n = 1 << 24
    if want("sst_fixed"):
        out = torch.empty(n, dtype=torch.int32, device=dev)
        t = timed(lambda: crc32c.batch_fixed(buf, 3992, 3988, n, out=out, mask=True), args.reps)
        report("sst_fixed", t, n * 3988, n * (3988 + 4), n)

    # SST-shaped, descriptors, with index spans (one per 64 MiB SST: 16 811 data spans)
    if want("sst_desc"):
        per = 16811
        files = n // (per + 122)
        offs, lns = [], []
        pos = 0
        for _ in range(files):
            offs.append(pos + np.arange(per, dtype=np.int64) * 3992)
            lns.append(np.full(per, 3988, dtype=np.int64))
            pos += per * 3992
            offs.append(np.array([pos], dtype=np.int64))
            lns.append(np.array([486977], dtype=np.int64))
            pos += 486977 + 4 + 3
            pos = (pos + 7) & ~7
        off = np.concatenate(offs)
        lens = np.concatenate(lns)
        assert off[-1] + lens[-1] + 4 <= buf.numel()
        d_off, d_len = torch.from_numpy(off).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev)
        out2 = torch.empty(len(off), dtype=torch.int32, device=dev)
        fn = lambda: crc32c.batch(buf, d_off, d_len, out=out2, mask=True, check_bounds=False)  # noqa: E731
        report("sst_desc", timed(fn, args.reps), lens.sum(), lens.sum() + 16 * len(lens), len(lens))
        ref = out2.clone()
        report("sst_desc_windows", timed(windows(fn), args.reps), lens.sum(), lens.sum() + 16 * len(lens), len(lens))
        res["sst_desc_windows"]["agrees"] = bool(torch.equal(ref, out2))
        # WriteRawBlock over the same blocks (MASK | WRITE_TRAILER into the trailer slots)
        fs = lambda: crc32c.batch(buf, d_off, d_len, out=out2, mask=True, trailer=True, check_bounds=False)  # noqa: E731
        report("sst_seal", timed(fs, args.reps), lens.sum(), lens.sum() + 20 * len(lens), len(lens))
        ref = out2.clone()
        report("sst_seal_windows", timed(windows(fs), args.reps), lens.sum(), lens.sum() + 20 * len(lens), len(lens))
        res["sst_seal_windows"]["agrees"] = bool(torch.equal(ref, out2))
        del d_off, d_len, out2

    # verify 4 KiB spans (fixed stride 4096, span 4092 B, trailer in the last 4 B)
    if want("verify_4k"):
        out = torch.empty(n, dtype=torch.int32, device=dev)
        mm = torch.empty(n, dtype=torch.uint8, device=dev)
        t = timed(lambda: crc32c.batch_fixed(buf, 4096, 4092, n, out=out, mismatch=mm, verify=True), args.reps)
        report("verify_4k", t, n * 4092, n * (4092 + 4 + 1 + 4), n)

    # adversarial
    m = 2 << 20
    lens = rng.integers(0, 70000, size=m).astype(np.int64)  # (drawn either way: the WAL image below
    off = np.sort(rng.integers(0, (16 << 30) - 70001, size=m)).astype(np.int64)  # comes from the same rng)
    if want("adversarial"):
        d_off, d_len = torch.from_numpy(off).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev)
        out3 = torch.empty(m, dtype=torch.int32, device=dev)
        fn = lambda: crc32c.batch(buf, d_off, d_len, out=out3, check_bounds=False)  # noqa: E731
        report("adversarial", timed(fn, args.reps), lens.sum(), lens.sum() + 16 * m, m)
        ref = out3.clone()
        report("adversarial_windows", timed(windows(fn), args.reps), lens.sum(), lens.sum() + 16 * m, m)
        res["adversarial_windows"]["agrees"] = bool(torch.equal(ref, out3))

        del d_off, d_len, out3

    # WAL: one 4 MiB log file of ~1 KB records written in log format, tiled
    from prismdb_amd import log

    file_bytes = 4 << 20
    nfiles = (16 << 30) // file_bytes
    img = build_log(rng, file_bytes)
    hoff, hlen = log.scan(img)
    buf[:nfiles * file_bytes].view(nfiles, file_bytes).copy_(torch.from_numpy(img).to(dev))
    base = np.arange(nfiles, dtype=np.int64)[:, None] * file_bytes
    all_off = (base + hoff.astype(np.int64)[None, :]).reshape(-1)
    all_len = np.tile(hlen.astype(np.int64), nfiles)
    d_hoff = torch.from_numpy(all_off).to(dev)
    d_hlen = torch.from_numpy(all_len.astype(np.int32)).to(dev)
    m = len(all_off)
    t = timed(lambda: log.seal_log(buf, d_hoff, d_hlen, check_bounds=False), args.reps)
    report("wal_seal", t, int(all_len.sum()) + m, int(all_len.sum()) + m * (1 + 4 + 12), m)
    d_soff, d_slen = d_hoff + 6, d_hlen + 1
    out4 = torch.empty(m, dtype=torch.int32, device=dev)
    mm4 = torch.empty(m, dtype=torch.uint8, device=dev)
    t = timed(lambda: crc32c.batch(buf, d_soff, d_slen, out=out4, mismatch=mm4, verify=True, log_header=True,
                                        check_bounds=False),
              args.reps)
    bad = int(mm4.sum())
    report("wal_verify", t, int(all_len.sum()) + m, int(all_len.sum()) + m * (1 + 4 + 1 + 12), m)
    res["wal_verify"]["mismatches"] = bad

    print(json.dumps({"reps": args.reps, "results": res}, indent=1))


def build_log(rng, nbytes):
    """A log file in LevelDB's record format (db/log_format.h), ~1 KB records
    (PrismDB YCSB WriteBatch: 980 B value + key + batch header), crc fields
    zero (sealed on the device), cut at nbytes."""
    import numpy as np

    B, H = 32768, 7
    out = bytearray()
    bo = 0
    while len(out) < nbytes:
        left = int(rng.integers(990, 1031))
        begin = True
        while True:
            if B - bo < H:
                out += bytes(B - bo)
                bo = 0
            frag = min(left, B - bo - H)
            end = frag == left
            typ = 1 if begin and end else 2 if begin else 4 if end else 3
            out += bytes(4) + bytes([frag & 0xFF, frag >> 8, typ]) + rng.bytes(frag)
            bo += H + frag
            left -= frag
            begin = False
            if left == 0:
                break
    img = np.frombuffer(bytes(out[:nbytes]), dtype=np.uint8).copy()
    return img


if __name__ == "__main__":
    main()
