#!/bin/bash
# span-kernel instruction mix on 16 Mi x 4 KiB descriptors after the scalar-state work
set -o pipefail
R=$(pwd)
bash tools/prof_desc.sh || exit $?
cd $R
python - <<'PY'
import csv, collections
for path in ["gpurun_out/pd_sq/run_counter_collection.csv", "gpurun_out/pd_sq2/run_counter_collection.csv"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "span_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in acc.items():
        print(c, round(max(d.values()) / (1 << 24), 2), "per span (largest dispatch)")
PY
grep -i "crc32c" gpurun_out/pd_kt/run_kernel_stats.csv | cut -c1-140
