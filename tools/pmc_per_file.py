#!/usr/bin/env python3
"""Summarise the per-file seal / verify profiles of the one-launch kernel
(tools/gpurun scripts running tools/run_file.py under rocprofv3: a kernel
trace with --stats, then FETCH_SIZE and WRITE_SIZE each in a pass of its own)
into one JSON: per-file kernel time, HBM bytes against the algorithmic bytes.

    python tools/pmc_per_file.py <gpurun_out dir> <prefix> <out.json>

<prefix>_{seal7,verify7,seal1,verify1}/{kt,fetch,write}/ are read.  HBM bytes
follow MI355X_MICROARCH.md: read = 2 x FETCH_SIZE KiB on gfx950 (128-B
requests tallied at 64 B), write = WRITE_SIZE KiB.  One file: 16 811 data
spans of 3988 B + the 486 977-B index span; algorithmic bytes per span =
len + 4 (trailer) + 12 (descriptor).
"""
import collections
import csv
import json
import os
import sys

ND, DATA, INDEX = 16811, 3988, 486977


def main():
    d, prefix, out = sys.argv[1], sys.argv[2], sys.argv[3]
    res = {"what": "one-launch kernel over 56 distinct SST files (16 811 x 3988 B @ 3992 + 486 977 B each), "
                   "1 or 7 files per call, seal (MASK|WRITE_TRAILER) vs verify; rocprofv3 --kernel-trace --stats "
                   "and --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/run_file.py 56 --files 56 "
                   "--per-call F [--verify]); read = 2 x FETCH_SIZE KiB (gfx950), write = WRITE_SIZE KiB",
           "runs": {}}
    for t in ("seal7", "verify7", "seal1", "verify1"):
        base = os.path.join(d, f"{prefix}_{t}")
        kern = "crc32c_direct_kernel<%s>" % ("true" if t.startswith("verify") else "false")
        st = None
        with open(os.path.join(base, "kt", "run_kernel_stats.csv")) as f:
            for r in csv.DictReader(f):
                if kern in r["Name"]:
                    st = {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
        c = {}
        for sub in ("fetch", "write"):
            acc = collections.defaultdict(list)
            with open(os.path.join(base, sub, "run_counter_collection.csv")) as f:
                for r in csv.DictReader(f):
                    if kern in r.get("Kernel_Name", ""):
                        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            c.update({k: sum(v) / len(v) for k, v in acc.items()})
        files = 7 if t.endswith("7") else 1
        spans = files * (ND + 1)
        algo = files * (ND * (DATA + 4 + 12) + INDEX + 4 + 12)
        rd, wr = 2 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        res["runs"][t] = {"kernel_trace": st, "files_per_call": files,
                          "us_per_file": round(st["avg_ns"] / 1000 / files, 2),
                          "algorithmic_bytes_per_call": algo, "hbm_read_bytes_per_call": rd,
                          "hbm_write_bytes_per_call": wr, "read_over_algorithmic": round(rd / algo, 4),
                          "write_bytes_per_span": round(wr / spans, 1),
                          "GBps_algorithmic": round(algo / st["avg_ns"], 1)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res["runs"].items():
        print(k, v["us_per_file"], "us/file", v["read_over_algorithmic"], "x read", v["write_bytes_per_span"],
              "B written/span", v["GBps_algorithmic"], "GB/s")


if __name__ == "__main__":
    main()
