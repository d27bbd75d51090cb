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
    "ring4_nt1": {"PRISMDB_RING": 4, "PRISMDB_NT_LOADS": 1},
    "ring4_nt0": {"PRISMDB_RING": 4, "PRISMDB_NT_LOADS": 0},
}


def do_build(names):
    from prismdb_amd.build import build

    for name in names:
        print(build(defines=VARIANTS[name], lib_path=os.path.join(VDIR, f"lib_{name}.so")))


def do_run(args, names):
    import torch

    from prismdb_amd import crc32c  # product lib: data generator

    dev = torch.device("cuda", 0)
    nblk = (args.gib << 30) // 4096
    buf = torch.empty(nblk * 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    stream = torch.cuda.current_stream()
    libs = {}
    for name in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"), mode=os.RTLD_LOCAL)
        f = lib.leveldb_crc32c_batch_fixed
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        libs[name] = f
    outs = {n: torch.empty(nblk, dtype=torch.int32, device=dev) for n in names}

    def call(n):
        rc = libs[n](buf.data_ptr(), 4096, 4096, nblk, 0, outs[n].data_ptr(), None, 0,
                     ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0, (n, rc)

    def timed(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        call(n)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3

    for n in names:
        timed(n)
    ref = outs[names[0]]
    same = {n: bool(torch.equal(outs[n], ref)) for n in names}
    res = {n: [] for n in names}
    for _ in range(args.reps):
        for n in names:
            res[n].append(timed(n))
    algo = nblk * 4100
    print(json.dumps({"gib": args.gib, "reps": args.reps, "identical_results": same,
                      "results": {n: {"GB/s_median": round(algo / statistics.median(v) / 1e9, 1),
                                      "GB/s_best": round(algo / min(v) / 1e9, 1),
                                      "ms_median": round(statistics.median(v) * 1e3, 3)}
                                  for n, v in res.items()}}, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--gib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    names = args.only or list(VARIANTS)
    if args.mode == "build":
        do_build(names)
    else:
        do_run(args, names)


if __name__ == "__main__":
    main()
