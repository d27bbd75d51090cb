#!/bin/bash
# single-exit fixed kernel: parity, then A/B of ring/run knobs (early6, run3, run7) and the no-fold ceiling
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s_tests.log 2>&1 && \
timeout -k 10 500 python tools/variants.py run --only base nofold early6 run3 run7 --gib 64 --reps 7 > gpurun_out/s_variants.json 2>gpurun_out/s_variants.err
rc=$?
tail -3 gpurun_out/s_tests.log
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/s_variants.json"))
    print(d["agree"])
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
