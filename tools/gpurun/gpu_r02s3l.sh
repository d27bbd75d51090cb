#!/bin/bash
# List kernel grid (one block per 1024 spans): WAL call A/B and kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base v3_bytes --work wal wal_seal --gib 32 --reps 7 > $O/s3l_variants.json 2> $O/s3l_variants.err || { tail -20 $O/s3l_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3l_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s3l_kt -o run --output-format csv -- python3 $R/tools/run_wal.py 3 > $O/s3l_kt.log 2>&1 || exit $?
cd $R && python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/s3l_kt/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "prismdb" in r["Name"] or "fill" in r["Name"]: print(r["Name"][:64], r["Calls"], r["AverageNs"])
PY
