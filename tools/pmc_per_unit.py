#!/usr/bin/env python3
"""Per-unit PMC summary of one kernel from tools/prof_*.sh output directories.

    python tools/pmc_per_unit.py <dir> <kernel substring> <units per dispatch> [--label L]

Averages every counter over the kernel's dispatches (rocprofv3 csv rows are
per dispatch and counter), divides by the units (records, blocks) one
dispatch processes, and adds the kernel-trace duration."""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("units", type=float)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (d, c), v in acc.items():
        per[c].append(sum(v))
    counters = {c: sum(v) / len(v) for c, v in per.items()}
    stats = {}
    p = os.path.join(a.dir, "kt", "run_kernel_stats.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            stats[r["Name"][:90]] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 1)}
    print(json.dumps({"label": a.label, "kernel": a.kernel, "units_per_dispatch": a.units,
                      "per_unit": {c: round(v / a.units, 2) for c, v in sorted(counters.items())},
                      "kernel_stats": stats}, indent=1))


if __name__ == "__main__":
    main()
