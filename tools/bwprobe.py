#!/usr/bin/env python3
"""HBM read-ceiling probes + engine kernel comparison (measurement support).

    python tools/bwprobe.py [--gib 16] [--reps 5]

Prints one JSON object: read bandwidth of a plain streaming XOR-fold kernel per
load width (4/8/16 B per lane), cache policy (default / nt) and grid size, and
the engine's fixed and generic kernels on the same 4 KiB-block buffer, all
interleaved in one process (cdna_hip_programming.md 5.4 rule 24).
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")  # the library's prismdb_* setters act only with this
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "tools", "_build", "libbwprobe.so")


def build():
    src = os.path.join(ROOT, "tools", "bwprobe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared",
                               src, "-o", SO])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--blocks-only", action="store_true", help="block-pattern probes + dword nt grid-stride only")
    args = ap.parse_args()
    build()
    import torch
    from prismdb_amd import crc32c
    from prismdb_amd._lib import lib

    probe = ctypes.CDLL(SO)
    probe.bwprobe_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    nbytes = args.gib << 30
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    out = torch.empty(8192 * 256, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3

    probe.bwprobe_blocks.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    variants = {}
    sp = ctypes.c_void_p(stream.cuda_stream)
    nb = nbytes // 4096
    for wg, grid in ((1024, 256), (256, 1024), (256, 2048)):
        for ring in (1, 2, 4):
            for xcd in (0, 1):
                key = f"blocks_wg{wg}_g{grid}_r{ring}_x{xcd}"
                variants[key] = (lambda w=wg, g=grid, r=ring, x=xcd: probe.bwprobe_blocks(
                    buf.data_ptr(), nb, out.data_ptr(), w, r, x, g, sp), nb * 4096)
    probe.bwprobe_blocks_store.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p]
    res_out = torch.empty(nb, dtype=torch.int32, device=dev)
    for mode in range(7):
        variants[f"blocks_store_mode{mode}"] = (lambda md=mode: probe.bwprobe_blocks_store(
            buf.data_ptr(), nb, res_out.data_ptr(), md, 256, sp), nb * 4096)
    probe.bwprobe_runs_store.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    for mode, params in ((0, (128, 256, 512)), (1, (2, 4, 8)), (2, (0,))):
        for prm in params:
            variants[f"runs_store_m{mode}_p{prm}"] = (lambda md=mode, pr=prm: probe.bwprobe_runs_store(
                buf.data_ptr(), nb, res_out.data_ptr(), md, pr, 256, sp), nb * 4096)
    for width in ((4,) if args.blocks_only else (4, 8, 16)):
        for nt in ((1,) if args.blocks_only else (0, 1)):
            for grid in (1024, 2048, 4096, 8192):
                key = f"read_w{width}_nt{nt}_g{grid}"
                variants[key] = (lambda w=width, t=nt, g=grid: probe.bwprobe_read(
                    buf.data_ptr(), nbytes, out.data_ptr(), w, t, g, ctypes.c_void_p(stream.cuda_stream)), nbytes)
    nblk = nbytes // 4096
    crc_out = torch.empty(nblk, dtype=torch.int32, device=dev)
    variants["crc_fixed_4k"] = (lambda: crc32c.batch_fixed(buf, 4096, 4096, nblk, out=crc_out), nblk * 4100)

    def generic():
        lib().prismdb_crc32c_force_generic(1)
        try:
            crc32c.batch_fixed(buf, 4096, 4096, nblk, out=crc_out)
        finally:
            lib().prismdb_crc32c_force_generic(0)
    lib().prismdb_crc32c_force_generic.argtypes = [ctypes.c_int]
    variants["crc_generic_4k"] = (generic, nblk * 4100)
    res = {k: [] for k in variants}
    for k, (fn, _) in variants.items():  # warm
        timed(fn)
    for _ in range(args.reps):
        for k, (fn, _) in variants.items():
            res[k].append(timed(fn))
    summary = {k: {"GB/s_median": round(variants[k][1] / statistics.median(v) / 1e9, 1),
                   "GB/s_best": round(variants[k][1] / min(v) / 1e9, 1),
                   "ms_median": round(statistics.median(v) * 1e3, 3)} for k, v in res.items()}
    print(json.dumps({"buffer_gib": args.gib, "reps": args.reps, "results": summary}, indent=1))


if __name__ == "__main__":
    main()
