#!/usr/bin/env python3
"""Read + fold probes for ~1 KB records (tools/recfold.hip; measurement support).

    python tools/recfold.py [--gib 16] [--reps 5]

Times the lane and octet read + fold structures of tools/recfold.hip over
the same buffer, interleaved, and prints GB/s of record bytes: would an octet
lane kernel (8 lanes per record) beat the one-record-per-lane one?
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "tools", "_build", "librecfold.so")


def build():
    src = os.path.join(ROOT, "tools", "recfold.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", src,
                               "-o", SO])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stride", type=int, default=1031)
    ap.add_argument("--len", type=int, default=1024)
    args = ap.parse_args()
    build()
    import torch

    lib = ctypes.CDLL(SO)
    lib.recfold.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    nbytes = args.gib << 30
    buf = torch.ones(nbytes, dtype=torch.uint8, device=dev)
    nrec = (nbytes - args.len - 256) // args.stride
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    out = torch.empty(nrec, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    # bytes of the lines that hold a record's bytes (what each mode reads from memory at least once)
    lines = sum(((s + args.len - 1) // 128 - s // 128 + 1) for s in range(0, args.stride * 128, args.stride)) / 128
    algo = nrec * args.len

    def timed(mode):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        rc = lib.recfold(buf.data_ptr(), nrec, args.stride, args.len, out.data_ptr(), mode, cus, sp)
        e1.record(stream)
        e1.synchronize()
        assert rc == 0
        return e0.elapsed_time(e1) / 1e3

    names = {0: "lane_fold", 2: "lane_fold_2ch", 3: "lane_fold_4ch", 1: "octet_fold"}
    for m in names:
        timed(m)
    res = {v: [] for v in names.values()}
    for rep in range(args.reps):
        for m in (list(names) if rep % 2 == 0 else list(names)[::-1]):
            res[names[m]].append(timed(m))
    print(json.dumps({"records": nrec, "len": args.len, "stride": args.stride, "lines_per_record": round(lines, 3),
                      "GBps_record_bytes": {k: round(algo / statistics.median(v) / 1e9, 1) for k, v in res.items()},
                      "roofline_frac": {k: round(algo / statistics.median(v) / 8e12, 4) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
