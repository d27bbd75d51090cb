#!/bin/bash
# A/B: quad kernel v1 (5b818f4) vs v2 (contiguous scalar reads, 32-bit window, vector geometry); then GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python tools/variants.py run --only quadv1 quadv2 --gib 16 --reps 8 > $O/r02f_variants.json 2> $O/r02f_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02f_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02f_tests.log 2>&1
rc=$?; tail -3 $O/r02f_tests.log; exit $rc
