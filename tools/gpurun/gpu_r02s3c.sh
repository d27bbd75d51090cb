#!/bin/bash
# Lane kernel (one log record per lane): GPU suite, smoke, A/B against the quad kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3c_tests.log 2>&1 || { tail -30 $O/s3c_tests.log; exit 1; }
tail -1 $O/s3c_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3c_smoke.log 2>&1 || { tail -20 $O/s3c_smoke.log; exit 1; }
tail -1 $O/s3c_smoke.log
timeout -k 10 600 python tools/variants.py run --only base quadk --work wal mixed desc4k --gib 32 --reps 5 > $O/s3c_variants.json 2> $O/s3c_variants.err || { tail -20 $O/s3c_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3c_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
