#!/bin/bash
# A/B: quad path for log batches only (base) vs every descriptor batch (quad_all) after the zero-area spread; GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only quadv2 base quad_all --gib 16 --reps 8 > $O/r02m_variants.json 2> $O/r02m_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02m_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02m_tests.log 2>&1
rc=$?; tail -3 $O/r02m_tests.log; exit $rc
