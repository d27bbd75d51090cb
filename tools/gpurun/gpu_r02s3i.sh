#!/bin/bash
# Lane kernel v3 (line-aligned body loads): GPU suite, smoke, A/B against lane v2 and the quad kernel, FETCH_SIZE
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3i_tests.log 2>&1 || { tail -30 $O/s3i_tests.log; exit 1; }
tail -1 $O/s3i_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3i_smoke.log 2>&1 || { tail -20 $O/s3i_smoke.log; exit 1; }
tail -1 $O/s3i_smoke.log
timeout -k 10 600 python tools/variants.py run --only base lane_v2 quadk --work wal --gib 32 --reps 5 > $O/s3i_variants.json 2> $O/s3i_variants.err || { tail -20 $O/s3i_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3i_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-include-regex crc32c_lane_kernel --pmc FETCH_SIZE -d $O/s3i_fetch -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/s3i_fetch.log 2>&1 || exit $?
cd $R && python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/s3i_fetch/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        print(r["Kernel_Name"][:50], r["Counter_Name"], r["Counter_Value"])
PY
