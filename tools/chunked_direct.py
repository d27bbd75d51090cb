#!/usr/bin/env python3
"""Probe: a large descriptor batch as consecutive one-launch calls of <= 2^17
spans each, against the planner path's single call (the path such batches
take today).  Measurement only, nothing in the product uses this split.

    python tools/chunked_direct.py [--reps 5]

Workloads (bench_configs.py's): sst_desc (3988-B spans at stride 3992, 16 Mi
spans, one 486 977-B index span per 16 811) and config3_mixed (1/4/16/64 KiB
spans back to back, ~16 GiB).  Windows: 2^17 spans (one-launch maximum) and
2^16; ordered, and flagged PRISMDB_CRC32C_UNORDERED (the windows are
disjoint: every other launch may overlap its predecessor).  Prints one JSON
object: ms and roofline fraction (L + 4 + 12 B per span over 8 TB/s) per
variant, and whether the results agree with the planner call.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    buf = torch.empty(64 << 30, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)

    def timed(fn):
        fn()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        return statistics.median(ts)

    rng = np.random.default_rng(0x5EED0003)
    ml = rng.choice([1024, 4096, 16384, 65536], size=(16 << 30) // 21760).astype(np.int64)
    mo = np.concatenate([[0], np.cumsum(ml)[:-1]])
    nd = 16811
    ns = 1 << 24
    per = nd + 1
    nf = ns // per
    so = np.zeros(nf * per, dtype=np.int64)
    sl = np.zeros(nf * per, dtype=np.int64)
    fbytes = nd * 3992 + 486977 + 3
    for f in range(nf):
        so[f * per:f * per + nd] = f * fbytes + np.arange(nd, dtype=np.int64) * 3992
        sl[f * per:f * per + nd] = 3988
        so[f * per + nd] = f * fbytes + nd * 3992
        sl[f * per + nd] = 486977
    work = {"sst_desc": (so, sl), "config3_mixed": (mo, ml)}
    res = {}
    for name, (o, ln) in work.items():
        d_off = torch.from_numpy(o).to(dev)
        d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
        n = len(o)
        algo = int(ln.sum()) + 16 * n
        ref = torch.empty(n, dtype=torch.int32, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        r = {"spans": n}
        t = timed(lambda: crc32c.batch(buf, d_off, d_len, out=ref, check_bounds=False))
        r["planner_one_call"] = {"ms": round(t * 1e3, 3), "roofline_frac": round(algo / t / 8e12, 4)}
        for win in (1 << 17, 1 << 16):
            for unordered in (False, True):
                def run():
                    for i in range(0, n, win):
                        j = min(n, i + win)
                        crc32c.batch(buf, d_off[i:j], d_len[i:j], out=out[i:j], check_bounds=False,
                                     unordered=unordered)
                out.zero_()
                t = timed(run)
                key = f"direct_windows_{win}" + ("_unordered" if unordered else "")
                r[key] = {"ms": round(t * 1e3, 3), "roofline_frac": round(algo / t / 8e12, 4),
                          "calls": (n + win - 1) // win, "agree": bool(torch.equal(out, ref))}
        res[name] = r
        del d_off, d_len, ref, out
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
