#!/bin/bash
# wave-parallel long-span combine: GPU suite + alternating A/B vs 2e80ac2 (+ huge 64 MiB spans)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bg_tests.log 2>&1 && \
timeout -k 10 500 python tools/variants.py run --only prev base --gib 64 --reps 12 > gpurun_out/bg_variants.json 2>gpurun_out/bg_variants.err
rc=$?
tail -3 gpurun_out/bg_tests.log
grep -E "FAILED|Error" gpurun_out/bg_tests.log | head -10
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/bg_variants.json"))
    print({k: v for k, v in d["agree"].items() if not v})
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
