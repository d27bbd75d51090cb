#!/usr/bin/env python3
"""Where a file-sized one-launch call spends its time, wave by wave.

Drives the `direct_ts` build of tools/variants.py (per-wave s_memrealtime
stamps written after the results: entry, descriptors in, tables in, first
fold, ring drained, exit) over one SST file's spans (16 811 x 3988 B @ 3992 +
the 486 977-B index span), 20 calls back to back, and prints the last call's
phase times in microseconds relative to the first wave's entry (entry,
descriptors in, tables in, slot 0's data in, first fold done, ring drained,
exit): percentiles
over the waves with a static run, and the latest exit of any wave.

    python tools/direct_timeline.py [--lib tools/vlib/lib_direct_ts.so] [--data-only]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "vlib", "lib_direct_ts.so"))
    ap.add_argument("--data-only", action="store_true", help="no index span")
    args = ap.parse_args()
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    lib = ctypes.CDLL(args.lib, mode=os.RTLD_LOCAL)
    g = lib.leveldb_crc32c_batch
    g.restype = ctypes.c_int
    g.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_void_p]
    nd = 16811
    buf = torch.empty(nd * 3992 + 486977 + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00F1)
    off = np.concatenate([np.arange(nd, dtype=np.int64) * 3992, [nd * 3992]])
    lens = np.array([3988] * nd + [486977], dtype=np.int32)
    if args.data_only:
        off, lens = off[:nd], lens[:nd]
    n = len(off)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    nwaves = 256 * 12
    base = (n + 3) & ~3
    out = torch.zeros(base + 2 * 8 * nwaves, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    for _ in range(20):
        rc = g(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, n, out.data_ptr(), None, 0,
               ctypes.c_void_p(s.cuda_stream))
        assert rc == 0
    torch.cuda.synchronize()
    ts = out[base:].cpu().numpy().view(np.uint64).reshape(nwaves, 8).astype(np.int64)
    live = ts[:, 0] != 0
    t0 = ts[live, 0].min()
    ts = ts[:, [0, 1, 2, 7, 3, 4, 5, 6]]  # entry, desc, tables, first wait, first fold, drained, exit, m
    rel = (ts[:, :7] - t0) / 100.0  # 100 MHz -> us
    run = live & (ts[:, 7] > 0)
    res = {"spans": n, "waves_with_stamps": int(live.sum()), "waves_with_run": int(run.sum()),
           "last_exit_us": float(rel[live, 6].max())}
    names = ["entry", "descriptors_in", "tables_in", "first_data_in", "first_fold_done", "ring_drained", "exit"]
    for k, name in enumerate(names):
        v = rel[run, k]
        v = v[ts[run, k] != 0]
        if len(v):
            res[name] = {p: round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)}
    # Where the drain spread lives: within a group (one CU's 12 waves), across
    # groups, or across XCDs (group g runs on XCD g % 8: workgroups are dealt
    # round-robin over the XCDs).
    g = np.arange(nwaves) // 12
    dr = rel[:, 5]
    ok = run & (ts[:, 5] != 0)
    gmax, gmin, gmean, xs = [], [], [], {x: [] for x in range(8)}
    for grp in np.unique(g[ok]):
        v = dr[ok & (g == grp)]
        gmax.append(v.max())
        gmin.append(v.min())
        gmean.append(v.mean())
        xs[int(grp) % 8].extend(v.tolist())
    gmax, gmin, gmean = np.array(gmax), np.array(gmin), np.array(gmean)
    res["drain_by_group"] = {
        "group_max": {p: round(float(np.percentile(gmax, p)), 2) for p in (0, 10, 50, 90, 100)},
        "group_mean": {p: round(float(np.percentile(gmean, p)), 2) for p in (0, 10, 50, 90, 100)},
        "within_group_range_mean": round(float((gmax - gmin).mean()), 2),
        "xcd_mean": [round(float(np.mean(xs[x])), 2) if xs[x] else None for x in range(8)],
        "wave_in_group_mean": [round(float(dr[ok & (np.arange(nwaves) % 12 == k)].mean()), 2) for k in range(12)],
    }
    m = ts[:, 7]
    res["drain_by_run_length"] = {int(k): round(float(dr[ok & (m == k)].mean()), 2) for k in np.unique(m[ok])}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
