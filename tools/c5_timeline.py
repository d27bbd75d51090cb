#!/usr/bin/env python3
"""One config-5 partition call, kernel by kernel (the planner path's lead-in
and tail around the pair-run kernel).

    python tools/c5_timeline.py run [calls] [variant]  # GPU box, under rocprofv3 --kernel-trace
                                                     # (variant: tools/vlib/lib_<variant>.so)
    python tools/c5_timeline.py parse <run_kernel_trace.csv>

`run` builds one partition of BASELINE config 5 (143 SST files x (16 811 x
3988 B @ 3992 + one 486 977-B index span) = 2 404 116 spans, as bench.py's
config5 legs) and issues `calls` sealing calls (MASK | WRITE_TRAILER) on one
stream, then `calls` verify calls.  `parse` prints, for the last sealing call
and the last verify call, every kernel from the call's first to its last as
CSV rows (start relative to the call's first kernel, duration, queue, name),
and the time outside the pair-run kernel: lead-in (call start to pair start)
and tail (pair end to call end)."""
import csv
import json
import os
import sys

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ND, DATA, STRIDE, INDEX = 16811, 3988, 3992, 486977
NFILES = 143


def run(calls, variant=None):
    import ctypes

    import numpy as np
    import torch

    from prismdb_amd import crc32c
    from prismdb_amd._lib import lib

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    fbytes = (ND * STRIDE + INDEX + 4 + 255) & ~255
    off1 = np.concatenate([np.arange(ND, dtype=np.int64) * STRIDE, [ND * STRIDE]])
    len1 = np.concatenate([np.full(ND, DATA, dtype=np.int64), [INDEX]])
    off = (np.arange(NFILES, dtype=np.int64)[:, None] * fbytes + off1[None, :]).reshape(-1)
    lens = np.tile(len1, NFILES)
    n = len(off)
    buf = torch.empty(NFILES * fbytes, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00C5)
    buf[torch.from_numpy(off + lens - 1).to(dev)] = 0
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    mm = torch.empty(n, dtype=torch.uint8, device=dev)
    if variant:  # a tools/variants.py build instead of the product library
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "vlib", f"lib_{variant}.so"), mode=os.RTLD_LOCAL)
        L.leveldb_crc32c_batch.restype = ctypes.c_int
        L.leveldb_crc32c_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                                                   ctypes.c_uint32, ctypes.c_void_p]
    else:
        L = lib()
    sp = torch.cuda.current_stream().cuda_stream
    for verify in (False, True):
        for _ in range(calls):
            rc = L.leveldb_crc32c_batch(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, n, out.data_ptr(),
                                        mm.data_ptr() if verify else None, 0 if verify else 3, sp)
            assert rc == 0, rc
        torch.cuda.synchronize()
    assert int(mm.sum().item()) == 0
    print(json.dumps({"spans": n, "calls": calls}))


def parse(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    res = {}
    # a call starts at a plan kernel (or the fill before it) and ends before the next call's first kernel
    starts = [i for i, r in enumerate(rows) if "crc32c_plan_kernel" in r["Kernel_Name"]]
    calls = []
    for j, i in enumerate(starts):
        b = i - 1 if i > 0 and "fillBuffer" in rows[i - 1]["Kernel_Name"] else i
        e = starts[j + 1] if j + 1 < len(starts) else len(rows)
        if j + 1 < len(starts) and "fillBuffer" in rows[e - 1]["Kernel_Name"]:
            e -= 1
        calls.append(rows[b:e])
    seal = [c for c in calls if any("crc32c_trailer_kernel" in r["Kernel_Name"] for r in c)]
    ver = [c for c in calls if c not in seal and any(k in r["Kernel_Name"] for r in c
                                                      for k in ("pair_kernel<true>", "bulk_kernel<true>"))]
    for name, group in (("seal", seal), ("verify", ver)):
        if not group:
            continue
        c = [r for r in group[-1] if "crc32c" in r["Kernel_Name"]]
        t0 = int(c[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in c)
        pair = [r for r in c if "crc32c_pair_kernel" in r["Kernel_Name"] or "crc32c_bulk_kernel" in r["Kernel_Name"]]
        print(f"# {name}: call {(t1 - t0) / 1e3:.1f} us")
        print("start_us,duration_us,queue,kernel")
        for r in c:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(s - t0) / 1e3:.1f},{(e - s) / 1e3:.1f},{r['Queue_Id']},{r['Kernel_Name'].split('(')[0]}")
        if pair:
            ps, pe = int(pair[0]["Start_Timestamp"]), int(pair[0]["End_Timestamp"])
            res[name] = {"call_us": round((t1 - t0) / 1e3, 1), "lead_in_us": round((ps - t0) / 1e3, 1),
                         "pair_us": round((pe - ps) / 1e3, 1), "tail_us": round((t1 - pe) / 1e3, 1),
                         "outside_pair_us": round((t1 - t0 - (pe - ps)) / 1e3, 1), "calls_seen": len(group)}
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 5, sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        parse(sys.argv[2])
