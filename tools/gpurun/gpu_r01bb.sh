#!/bin/bash
# alternating-order harness: A/A (prev, prevcopy) and refactor (base) vs 8c67c37
set -o pipefail
mkdir -p gpurun_out

timeout -k 10 500 python tools/variants.py run --only prev prevcopy base --gib 64 --reps 16 > gpurun_out/bb_variants.json 2>gpurun_out/bb_variants.err
rc=$?
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/bb_variants.json"))
    print({k: v for k, v in d["agree"].items() if not v})
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
