#!/bin/bash
# Quad kernel (short records) first GPU run: GPU suite, then the secondary workloads.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02d_tests.log 2>&1
rc=$?; tail -30 $O/r02d_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python tools/bench_configs.py --reps 5 > $O/r02d_configs.json 2> $O/r02d_configs.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02d_configs.json"))
for k, v in d["results"].items():
    print(k, {x: v[x] for x in v if x in ("GiB/s", "roofline_frac", "ms", "mismatches")})
PY
exit $rc
