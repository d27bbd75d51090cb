#!/bin/bash
# span-kernel instruction mix on 16 Mi x 4 KiB descriptors (desc4k), for the generic-path gap
set -o pipefail
R=$(pwd)
bash tools/prof_desc.sh || exit $?
cd $R
python - <<'PY'
import csv, collections
for name, path in [("span", "gpurun_out/pd_sq/run_counter_collection.csv"), ("span2", "gpurun_out/pd_sq2/run_counter_collection.csv")]:
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[(r["Kernel_Name"][:45], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(name, k, round(sum(v) / len(v), 1), round(sum(v) / len(v) / (1 << 24), 2), "per span")
PY
grep -i "crc32c" gpurun_out/pd_kt/run_kernel_stats.csv | cut -c1-160
