#!/usr/bin/env python3
"""Per-wave entry/exit times of the pair-run kernel on a bulk SST batch.

Drives the `pair_ts` build of tools/variants.py (each wave writes its entry
and exit s_memrealtime stamps after the results) over 16.6 M SST spans
(3988 B at stride 3992, one 486 977-B index span per 16 811), 3 calls, and
prints for the last call: exit times (us from the first entry) by
percentile, and the mean exit of each wave slot of a group (wave % 16: a
CU's four SIMDs hold four waves each, slot // 4 is a wave's age rank on its
SIMD).

    python tools/wave_timeline.py [--lib tools/vlib/lib_pair_ts.so] [--spans N]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")  # the library's prismdb_* setters act only with this


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "vlib", "lib_pair_ts.so"))
    ap.add_argument("--spans", type=int, default=1 << 24)
    ap.add_argument("--work", choices=["sst", "fixed", "mixed", "wal"], default="sst",
                    help="sst: SST descriptors (pair-run kernel); fixed: 16 Mi x 4 KiB fixed blocks (fixed kernel); "
                         "mixed: config 3's 1/4/16/64 KiB spans, 32 GiB (span kernel); "
                         "wal: ~1 KB log records, 16 GiB, LOG_HEADER verify (lane kernel, 8 waves per CU)")
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
    f = lib.leveldb_crc32c_batch_fixed
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    nd, stride, dl, il = 16811, 3992, 3988, 486977
    files = max(1, args.spans // (nd + 1))
    fb = nd * stride + il + 4
    off1 = np.concatenate([np.arange(nd, dtype=np.int64) * stride, [nd * stride]])
    len1 = np.concatenate([np.full(nd, dl, dtype=np.int64), [il]])
    off = (np.arange(files, dtype=np.int64)[:, None] * fb + off1[None, :]).reshape(-1)
    lens = np.tile(len1, files)
    n = len(off)
    if args.work == "fixed":
        n = args.spans
        off, lens = off[:1], lens[:1]
    elif args.work == "mixed":
        rng = np.random.default_rng(0x5EED0003)
        lens = rng.choice([1024, 4096, 16384, 65536], size=(32 << 30) // 21760).astype(np.int64)
        off = np.concatenate([[0], np.cumsum(lens)[:-1]])
        n = len(off)
    flags, wpc = 0, 16
    if args.work == "wal":
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from bench_configs import build_log
        from prismdb_amd import log

        fbl = 4 << 20
        img = build_log(np.random.default_rng(0x5EED0003), fbl)
        hoff, hlen = log.scan(img)
        nf = (16 << 30) // fbl
        off = ((np.arange(nf, dtype=np.int64)[:, None] * fbl + hoff.astype(np.int64)[None, :]) + 6).reshape(-1)
        lens = np.tile(hlen.astype(np.int64) + 1, nf)
        n = len(off)
        flags, wpc = 0x4, 8
    buf = torch.empty(max(files * fb, n * 4096 if args.work != "wal" else 16 << 30) + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    if args.work == "wal":
        buf[:nf * fbl].view(nf, fbl).copy_(torch.from_numpy(img).to(dev))
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nwaves = cus * wpc
    base = (n + 3) & ~3
    out = torch.zeros(base + 4 * nwaves, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    for _ in range(3):
        if args.work == "fixed":
            rc = f(buf.data_ptr(), 4096, 4096, n, 0, out.data_ptr(), None, 0, ctypes.c_void_p(s.cuda_stream))
        else:
            rc = g(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, n, out.data_ptr(), None, flags,
                   ctypes.c_void_p(s.cuda_stream))
        assert rc == 0
    torch.cuda.synchronize()
    ts = out[base:].cpu().numpy().view(np.uint64).reshape(nwaves, 2).astype(np.int64)
    live = ts[:, 0] != 0
    t0 = ts[live, 0].min()
    rel = (ts - t0) / 100.0
    ex = rel[live, 1]
    slot = (np.arange(nwaves) % wpc)[live]
    res = {"work": args.work, "spans": n, "waves": int(live.sum()),
           "entry": {p: round(float(np.percentile(rel[live, 0], p)), 1) for p in (0, 50, 100)},
           "exit": {p: round(float(np.percentile(ex, p)), 1) for p in (0, 10, 50, 90, 100)},
           "exit_by_slot": [round(float(ex[slot == k].mean()), 1) for k in range(wpc)],
           "exit_by_xcd": [round(float(ex[((np.arange(nwaves) // wpc)[live] % 8) == x].mean()), 1) for x in range(8)]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
