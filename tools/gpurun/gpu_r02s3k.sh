#!/bin/bash
# Lane kernel: one unaligned dword store per sealed header (vs four byte stores): GPU suite, smoke, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3k_tests.log 2>&1 || { tail -30 $O/s3k_tests.log; exit 1; }
tail -1 $O/s3k_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3k_smoke.log 2>&1 || { tail -20 $O/s3k_smoke.log; exit 1; }
tail -1 $O/s3k_smoke.log
timeout -k 10 600 python tools/variants.py run --only base v3_bytes --work wal wal_seal --gib 32 --reps 5 > $O/s3k_variants.json 2> $O/s3k_variants.err || { tail -20 $O/s3k_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3k_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
export TMPDIR=/tmp
