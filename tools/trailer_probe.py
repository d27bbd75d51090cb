#!/usr/bin/env python3
"""What 2.4 M scattered trailer stores cost on their own (the planner path's
trailer pass, crc32c_trailer_kernel, on a config-5 partition).

    python tools/trailer_probe.py        # GPU box; one JSON object

On a buffer of 143 SST files' size (9.6 GB, past the 256 MB MALL), with
hipEvents around each of `reps` launches (median, us):
  scatter4_c5      2 404 116 dword stores at the config-5 trailer positions
                   (16 811 at stride 3992 + the index's, per 67.6 MB file;
                   here uniformly: stride 3992, offset 3988)
  sector32_c5      the same lines, each a whole aligned 32-B sector
  scatter4_dense   the same count of dword stores, contiguous (no partial lines)
  trailer_pass     the product's own pass over the same trailers
                   (leveldb_crc32c_batch sealing: its trailer kernel is timed
                   by rocprof, not here) -- see tools/c5_timeline.py
Scattered partial-line writes cost the memory a read and a write each
(ECC words are written whole); whole sectors skip the read."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "probe_lib", "libfloor_probe.so")


def main():
    import numpy as np
    import torch

    dev = torch.device("cuda", 0)
    P = ctypes.CDLL(PROBE, mode=os.RTLD_LOCAL)
    vp = ctypes.c_void_p
    u32 = ctypes.c_uint32
    P.probe_sector.argtypes = [vp, u32, u32, u32, vp]
    P.probe_scatter_at.argtypes = [vp, u32, u32, u32, vp]
    n = 2404116
    stride = 3992
    buf = torch.zeros(n * stride + 4096, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    reps = 20

    def timed(fn):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(s)
            fn()
            b.record(s)
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
        return {"median_us": round(t[len(t) // 2], 1), "min_us": round(t[0], 1),
                "Gstores_per_s": round(n / t[len(t) // 2] / 1e3, 2)}

    b = ctypes.c_void_p(buf.data_ptr())
    res = {"stores": n, "buffer_GB": round(buf.numel() / 1e9, 2)}
    res["scatter4_c5"] = timed(lambda: P.probe_scatter_at(b, n, stride, 3988, sp))
    res["sector32_c5"] = timed(lambda: P.probe_sector(b, n, stride, 3988, sp))
    res["scatter4_dense"] = timed(lambda: P.probe_scatter_at(b, n, 4, 0, sp))
    res["scatter4_stride64"] = timed(lambda: P.probe_scatter_at(b, n, 64, 0, sp))
    res["sector32_stride64"] = timed(lambda: P.probe_sector(b, n, 64, 0, sp))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
