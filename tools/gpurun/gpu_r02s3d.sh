#!/bin/bash
# Lane kernel profile on WAL verify: kernel trace + PMC passes (tools/prof_quad.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
bash tools/prof_quad.sh s3d_lane crc32c_lane_kernel || exit $?
cd $R
python - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/s3d_lane/kt/*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:60], r["Calls"], r["AverageNs"], r["Percentage"])
for sub in ("sq", "sq2", "sq3", "fetch"):
    for f in glob.glob(f"gpurun_out/s3d_lane/{sub}/*counter_collection.csv"):
        acc = {}
        for r in csv.DictReader(open(f)):
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        print(sub, {k: round(sum(v) / max(1, len(set([0])) ), 0) for k, v in acc.items()})
PY
