#!/usr/bin/env python3
"""Compare compile-time variants of the engine in ONE process, interleaved.

    python tools/variants.py build                 # here: build tools/_build/variants/*.so
    python tools/variants.py run [--gib 64]        # GPU box: time them on one buffer

Each variant is the full library built with different -D knobs, loaded with
RTLD_LOCAL and driven through its own C ABI (leveldb_crc32c_batch_fixed) on the
same device buffer of 4 KiB blocks.  Results are also checked for equality.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "tools", "_build", "variants")

VARIANTS = {
    "base": {"PRISMDB_RING": 4, "PRISMDB_NT_LOADS": 1},
    # measurement-only: fixed kernel without the CRC fold (loads + stores), wrong results
    "nofold": {"PRISMDB_FIXED_NOFOLD": 1},
    "nofold_nt0": {"PRISMDB_FIXED_NOFOLD": 1, "PRISMDB_NT_LOADS": 0},
    "nostore": {"PRISMDB_FIXED_NOSTORE": 1},
    "nofold_nostore": {"PRISMDB_FIXED_NOFOLD": 1, "PRISMDB_FIXED_NOSTORE": 1},
    # measurement-only: span kernel folds rounds >= 12 / none (wrong results): the
    # ceiling of skipping chunk 0's padding rounds on ~1 KB spans
    "span_j12": {"PRISMDB_SPAN_J0": 12},
    "span_j16": {"PRISMDB_SPAN_J0": 16},
    # measurement-only: initial register always in round 0 (wrong where pad >= 64);
    # snop: the s_nop 4 before the span kernel's buffer loads, as it was
    "inj0": {"PRISMDB_SPAN_INJ0": 1},
    # log-record kernel without the padding-round skip (straight 16-round fold)
    "noskip": {"PRISMDB_LOG_ROUNDSKIP": 0},
    "snop": {"PRISMDB_SPAN_SNOP": 1},
    # fixed kernel: runs of 16 spans per wave instead of 64
    "run3": {"PRISMDB_RUN_LG": 3},
    # quad kernel (short records): measurement-only cuts (wrong results) and
    # the realignment lookups in 2 groups / 1 group instead of 4
    "quad_norealign": {"PRISMDB_QUAD_NOREALIGN": 1},
    "quad_nomask": {"PRISMDB_QUAD_NOMASK": 1},
    "quad_ra2": {"PRISMDB_QUAD_RALIGN_GROUPS": 2},
    "quad_ra1": {"PRISMDB_QUAD_RALIGN_GROUPS": 1},
    # quad kernel body loads: three address VALUs per load (clamped index)
    "quad_clamped": {"PRISMDB_QUAD_CLAMPED": 1},
    # quad kernel: unaligned body loads from the record's first byte (no head product)
    "quad_unaligned": {"PRISMDB_QUAD_UNALIGNED": 1},
    # (A/B helper: built from an older kernel source copied into the tree)
    "older_src": {"PRISMDB_OLDER_SRC": 1},
    # span kernel: initial register folded in (no ring-register copies at the merge)
    "inj_fold": {"PRISMDB_SPAN_INJ_RING": 0},
    # measurement-only: span kernel waits for every record's scalar read right away
    "rec_wait": {"PRISMDB_SPAN_REC_WAIT": 1},
    # measurement-only: fixed kernel with extra SALU / VALU per span pair (issue sensitivity)
    "salu200": {"PRISMDB_FIXED_DUMMY_SALU": 200},
    # span kernel: every group loads the tables, streams or not (as in round 1)
    "no_wg_exit": {"PRISMDB_SPAN_WG_EXIT": 0},
    # measurement-only: span kernel without its edge-byte load (desc4k stays exact: no tails)
    "noedge": {"PRISMDB_SPAN_NOEDGE": 1, "PRISMDB_MEASURE_ONLY": 1},
    # measurement: fixed kernel pairs spans half a run apart, like the span kernel's two streams
    "far_pair": {"PRISMDB_FIXED_FAR_PAIR": 1},
    # measurement: fixed kernel folds a pair as ONE dependent chain of 2K rounds (wrong results)
    "chain": {"PRISMDB_FIXED_CHAIN": 1, "PRISMDB_MEASURE_ONLY": 1},
    # fixed kernel: a pair's loads issued at wave priority 1 / 3 (s_setprio)
    "setprio1": {"PRISMDB_FIXED_SETPRIO": 1},
    "setprio3": {"PRISMDB_FIXED_SETPRIO": 3},
    # span kernel: streams in their own runs even when every record is one task (round 1)
    "no_pair_runs": {"PRISMDB_SPAN_PAIR_RUNS": 0},
    # planner: a long span's thread writes its segment records alone (as in round 1)
    "plan_serial": {"PRISMDB_PLAN_SERIAL_SEG": 1},
    "valu64": {"PRISMDB_FIXED_DUMMY_VALU": 64},
    # every descriptor batch through the quad kernel first
    "quad_all": {"PRISMDB_QUAD_DEFAULT": 1},
    # span kernel: at least 64 / 256 slices per record stream (finer tail balance)
    "slices64": {"PRISMDB_SLICES_PER_STREAM": 64},
    "slices256": {"PRISMDB_SLICES_PER_STREAM": 256},
    # task-balanced slices: ceil(T / 2^lg) of them (round 1) instead of exactly m per stream
    "slices_pow2": {"PRISMDB_SLICE_EXACT": 0},
    # span kernel runs of 2^lg records (before the exact partition)
    "runs_pow2": {"PRISMDB_RUNS_EXACT": 0},
    # span kernel runs mode (one-task records): 16 runs per stream (round 1) / 256
    "runs16": {"PRISMDB_RUNS_PER_STREAM": 16},
    "runs256": {"PRISMDB_RUNS_PER_STREAM": 256},
    # log batches through the quad kernel (four records per wave) instead of the lane kernel
    "quadk": {"PRISMDB_LANE_KERNEL": 0},
    # measurement-only: lane kernel loads without the fold (wrong results); the
    # alignment / nt probes of profiles/r02s3f, r02s3h were knobs of earlier lane-kernel builds
    "lane_nofold": {"PRISMDB_LANE_NOFOLD": 1, "PRISMDB_MEASURE_ONLY": 1},
    # lane kernel with 8 / 4 waves per CU (fewer record lines in flight per CU)
    "lane_w8": {"PRISMDB_LANE_THREADS": 512},
    "lane_w12": {"PRISMDB_LANE_THREADS": 768},
    "lane_w6": {"PRISMDB_LANE_THREADS": 384},
    "lane_w10": {"PRISMDB_LANE_THREADS": 640},
    "lane_w16": {"PRISMDB_LANE_THREADS": 1024},
    "lane_w4": {"PRISMDB_LANE_THREADS": 256},
    # quad kernel ring depth (tasks in flight + 1)
    "quad_r2": {"PRISMDB_QUAD_RING": 2},
    "quad_r3": {"PRISMDB_QUAD_RING": 3},
}
# Measured and dropped (profiles/r01_variants_ring_runs.json): refilling a ring
# pair before its fold with a 6-buffer ring ("early6") was no faster.
# Libraries built elsewhere (e.g. from an older commit in a git worktree) and
# dropped into VDIR as lib_<name>.so join the comparison with --only <name>.


def do_build(names):
    from prismdb_amd.build import build

    for name in names:
        if name not in VARIANTS:
            continue
        print(build(defines=VARIANTS[name], lib_path=os.path.join(VDIR, f"lib_{name}.so")))


def do_run(args, names):
    import numpy as np
    import torch

    from prismdb_amd import crc32c  # product lib: data generator

    dev = torch.device("cuda", 0)
    nblk = (args.gib << 30) // 4096
    buf = torch.empty(nblk * 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    libs = {}
    for name in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"), mode=os.RTLD_LOCAL)
        f = lib.leveldb_crc32c_batch_fixed
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        g = lib.leveldb_crc32c_batch
        g.restype = ctypes.c_int
        g.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        libs[name] = (f, g)
    out = torch.empty(nblk, dtype=torch.int32, device=dev)
    mm = torch.empty(nblk, dtype=torch.uint8, device=dev)
    off4k = torch.arange(nblk, dtype=torch.int64, device=dev) * 4096
    len4k = torch.full((nblk,), 4096, dtype=torch.int32, device=dev)
    rng = np.random.default_rng(0x5EED0003)
    ml = rng.choice([1024, 4096, 16384, 65536], size=(args.gib << 30) // 21760 // 2).astype(np.int64)
    mo = np.concatenate([[0], np.cumsum(ml)[:-1]])
    moff, mlen = torch.from_numpy(mo).to(dev), torch.from_numpy(ml.astype(np.int32)).to(dev)
    # WAL records (~1 KB, log format) tiled over the buffer, verified with LOG_HEADER
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_configs import build_log
    from prismdb_amd import log

    fb = 4 << 20
    nf = (args.gib << 30) // fb // 4
    img = build_log(rng, fb)
    hoff, hlen = log.scan(img)
    buf[:nf * fb].view(nf, fb).copy_(torch.from_numpy(img).to(dev))
    woff = torch.from_numpy(((np.arange(nf, dtype=np.int64)[:, None] * fb + hoff.astype(np.int64)[None, :]) + 6)
                            .reshape(-1)).to(dev)
    wlen = torch.from_numpy(np.tile(hlen.astype(np.int32) + 1, nf)).to(dev)
    nw = woff.numel()
    crc32c.batch(buf, woff, wlen, mask=True, trailer=True, log_header=True)  # log::Writer's header crcs
    wout = torch.empty(nw, dtype=torch.int32, device=dev)
    wmm = torch.empty(nw, dtype=torch.uint8, device=dev)
    # SST data blocks through descriptors: 3988-B spans (contents + type) at stride 3992
    ns = (args.gib << 30) // 3992 - 1
    soff = torch.arange(ns, dtype=torch.int64, device=dev) * 3992
    slen = torch.full((ns,), 3988, dtype=torch.int32, device=dev)
    sout = torch.empty(ns, dtype=torch.int32, device=dev)
    # huge spans: 256 x (64 MiB - 5 B) at odd offsets, 2048 segments each (split path + combine)
    nh = min(256, (args.gib << 30) // (64 << 20) - 1)
    hoff_ = torch.arange(nh, dtype=torch.int64, device=dev) * (64 << 20) + 1
    hlen_ = torch.full((nh,), (64 << 20) - 5, dtype=torch.int32, device=dev)
    hout = torch.empty(nh, dtype=torch.int32, device=dev)
    al = rng.integers(0, 70000, size=(args.gib << 30) // 35000 // 2).astype(np.int64)
    ao = np.sort(rng.integers(0, (args.gib << 30) // 2 - 70001, size=len(al))).astype(np.int64)
    aoff, alen = torch.from_numpy(ao).to(dev), torch.from_numpy(al.astype(np.int32)).to(dev)
    # one SST file's worth (16 811 data blocks + the 486 977-B index span), the
    # granularity a compaction verifies at: per-call latency, 50 calls per timing
    nfd = 16811
    foff = torch.from_numpy(np.concatenate([np.arange(nfd, dtype=np.int64) * 3992, [nfd * 3992]])).to(dev)
    flen = torch.from_numpy(np.concatenate([np.full(nfd, 3988, dtype=np.int32), [486977]]).astype(np.int32)).to(dev)
    fout = torch.empty(nfd + 1, dtype=torch.int32, device=dev)
    calls = {"file_fixed": 50, "file_desc": 50}
    work = {
        "fixed4k": (lambda n: libs[n][0](buf.data_ptr(), 4096, 4096, nblk, 0, out.data_ptr(), None, 0, sp),
                    nblk * 4100),
        "desc4k": (lambda n: libs[n][1](buf.data_ptr(), off4k.data_ptr(), len4k.data_ptr(), None, nblk,
                                        out.data_ptr(), None, 0, sp), nblk * 4112),
        "verify4k": (lambda n: libs[n][0](buf.data_ptr(), 4096, 4092, nblk, 0, out.data_ptr(), mm.data_ptr(), 0,
                                          sp), nblk * 4105),
        "mixed": (lambda n: libs[n][1](buf.data_ptr(), moff.data_ptr(), mlen.data_ptr(), None, len(ml),
                                       out.data_ptr(), None, 0, sp), int(ml.sum()) + 16 * len(ml)),
        "wal": (lambda n: libs[n][1](buf.data_ptr(), woff.data_ptr(), wlen.data_ptr(), None, nw,
                                     wout.data_ptr(), wmm.data_ptr(), 0x4, sp),
                int(hlen.sum() + len(hlen)) * nf + nw * (4 + 1 + 12)),
        # log::Writer's header crcs, sealed in place (the same bytes: the buffer does not change)
        "wal_seal": (lambda n: libs[n][1](buf.data_ptr(), woff.data_ptr(), wlen.data_ptr(), None, nw,
                                          wout.data_ptr(), None, 0x7, sp),
                     int(hlen.sum() + len(hlen)) * nf + nw * (4 + 4 + 12)),
        "sst3988": (lambda n: libs[n][1](buf.data_ptr(), soff.data_ptr(), slen.data_ptr(), None, ns,
                                         sout.data_ptr(), None, 0, sp), ns * (3988 + 4 + 12)),
        "huge64m": (lambda n: libs[n][1](buf.data_ptr(), hoff_.data_ptr(), hlen_.data_ptr(), None, nh,
                                         hout.data_ptr(), None, 0, sp), nh * ((64 << 20) - 5 + 16)),
        "adversarial": (lambda n: libs[n][1](buf.data_ptr(), aoff.data_ptr(), alen.data_ptr(), None, len(al),
                                             out.data_ptr(), None, 0, sp), int(al.sum()) + 16 * len(al)),
        "file_fixed": (lambda n: libs[n][0](buf.data_ptr(), 3992, 3988, nfd, 0, fout.data_ptr(), None, 0, sp),
                       nfd * (3988 + 4)),
        "file_desc": (lambda n: libs[n][1](buf.data_ptr(), foff.data_ptr(), flen.data_ptr(), None, nfd + 1,
                                           fout.data_ptr(), None, 0, sp), nfd * (3988 + 16) + 486977 + 16),
    }

    def timed(fn, n, k=1):  # mean of k back-to-back calls
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            rc = fn(n)
            assert rc == 0, (n, rc)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / k

    if args.work:
        work = {w: v for w, v in work.items() if w in args.work}
    res = {w: {n: [] for n in names} for w in work}
    agree = {}
    outs_of = {"wal": wout, "wal_seal": wout, "sst3988": sout, "huge64m": hout, "file_fixed": fout, "file_desc": fout}
    for w, (fn, _) in work.items():
        ref = None
        for n in names:
            o = outs_of.get(w, out)
            o.fill_(0)
            timed(fn, n)
            got = o.clone()
            if ref is None:
                ref = got
            agree[f"{w}:{n}"] = bool(torch.equal(ref, got))
        if w == "wal":
            agree["wal:no_mismatch"] = int(wmm.sum()) == 0
    # The order alternates every rep: a variant run right after another on the
    # same workload was measured up to 2 % faster than the same library run
    # first (an A/A run of one library under two names,
    # profiles/r01_variants_aa_position_bias.json), e.g. descriptor arrays left
    # in the 256 MB Infinity Cache by the first run.
    for rep in range(args.reps):
        for w, (fn, _) in work.items():
            for n in (names if rep % 2 == 0 else names[::-1]):
                res[w][n].append(timed(fn, n, calls.get(w, 1)))
    print(json.dumps({"gib": args.gib, "reps": args.reps, "agree": agree,
                      "results": {w: {n: {"GB/s_median": round(work[w][1] / statistics.median(v) / 1e9, 1),
                                          "ms_median": round(statistics.median(v) * 1e3, 4)}
                                      for n, v in r.items()} for w, r in res.items()}}, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--gib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--work", nargs="*", help="workloads to time (default: all)")
    args = ap.parse_args()
    names = args.only or list(VARIANTS)
    if args.mode == "build":
        do_build(names)
    else:
        do_run(args, names)


if __name__ == "__main__":
    main()
