#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of the bench into profiles/<tag>_pmc.json.

    python tools/pmc_summary.py <gpurun_out dir> <tag> [--kernel crc32c_fixed] [--nblocks N]

Inputs (written by tools/profile.sh on the GPU box):
  prof_kt/run_kernel_stats.csv          rocprofv3 --kernel-trace --stats
  prof_fetch/run_counter_collection.csv --pmc FETCH_SIZE      (own pass)
  prof_write/run_counter_collection.csv --pmc WRITE_SIZE      (own pass)
  prof_sq*/run_counter_collection.csv   SQ / GRBM counters    (own passes)

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide
coalesced streaming read (128-B requests tallied at 64 B), so the read side is
2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is taken as is.  The factor is
checked against the algorithmic byte count in the output ("fetch_ratio").
"""
import argparse
import collections
import csv
import json
import os


def counters(path, kernel):
    if not os.path.exists(path):
        return {}
    acc = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    # one row per dispatch and counter (already summed over XCDs/instances)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="crc32c_fixed")
    ap.add_argument("--nblocks", type=int, default=1 << 24)
    ap.add_argument("--block", type=int, default=4096)
    args = ap.parse_args()
    d = args.outdir
    stats = {}
    p = os.path.join(d, "prof_kt", "run_kernel_stats.csv")
    if os.path.exists(p):
        with open(p) as f:
            for r in csv.DictReader(f):
                if args.kernel in r["Name"]:
                    stats = {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                             "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    c = {}
    for sub in sorted(os.listdir(d)):
        if sub.startswith("prof_") and sub != "prof_kt":
            c.update(counters(os.path.join(d, sub, "run_counter_collection.csv"), args.kernel))
    algo = args.nblocks * (args.block + 4)
    out = {"tag": args.tag, "kernel": stats.get("name", args.kernel), "nblocks": args.nblocks,
           "algorithmic_bytes_per_launch": algo, "kernel_trace": stats, "counters": c}
    if "FETCH_SIZE" in c:
        read = 2.0 * c["FETCH_SIZE"] * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        out["hbm_read_bytes_per_launch"] = read
        out["hbm_write_bytes_per_launch"] = write
        out["hbm_bytes_per_launch"] = int(read + write)
        out["fetch_ratio"] = round(read / (args.nblocks * args.block), 4)
        out["correction"] = "read = 2 x FETCH_SIZE KiB (gfx950 half-count of 128-B requests), write = WRITE_SIZE KiB"
        if stats:
            out["hbm_GBps_from_pmc"] = round((read + write) / stats["avg_ns"], 1)
    if "GRBM_GUI_ACTIVE" in c and stats:
        out["effective_clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / stats["avg_ns"], 3)
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                out.setdefault("wave_cycle_shares", {})[k] = round(c[k] / wc, 3)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
        if k in c:
            out.setdefault("instructions_per_block", {})[k] = round(c[k] / args.nblocks, 1)
    os.makedirs("profiles", exist_ok=True)
    path = os.path.join("profiles", f"{args.tag}_pmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
