#!/bin/bash
# Lane kernel: side loads only where needed in the verify kernel, every task in the sealing kernel: GPU suite + smoke, A/B, PMC, secondary workloads
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3x_tests.log 2>&1 || { tail -30 $O/s3x_tests.log; exit 1; }
tail -1 $O/s3x_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3x_smoke.log 2>&1 || { tail -20 $O/s3x_smoke.log; exit 1; }
tail -1 $O/s3x_smoke.log
timeout -k 10 600 python tools/variants.py run --only base side_every --work wal wal_seal --gib 32 --reps 5 > $O/s3x_variants.json 2> $O/s3x_variants.err || { tail -20 $O/s3x_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3x_variants.json"))
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
bash tools/prof_quad.sh s3x_lane crc32c_lane_kernel || exit $?
cd $R
timeout -k 10 600 python tools/bench_configs.py > $O/s3x_configs.json 2> $O/s3x_configs.err || { tail -20 $O/s3x_configs.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3x_configs.json"))
for w, r in d["results"].items():
    print(w, {k: v for k, v in r.items() if k in ("GiB/s", "roofline_frac", "mismatches")})
PY
