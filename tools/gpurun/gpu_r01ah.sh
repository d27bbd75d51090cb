#!/bin/bash
# padding-round skip only in the LOG_HEADER span kernel: parity suite, A/B vs aa4ceca (prev)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/ah_tests.log 2>&1 && \
timeout -k 10 500 python tools/variants.py run --only prev base --gib 64 --reps 7 > gpurun_out/ah_variants.json 2>gpurun_out/ah_variants.err
rc=$?
tail -3 gpurun_out/ah_tests.log
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/ah_variants.json"))
    print(d["agree"])
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
