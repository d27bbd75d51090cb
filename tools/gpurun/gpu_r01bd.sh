#!/bin/bash
# alternating-order harness: session start (0c3382f), 044b212, HEAD
set -o pipefail
mkdir -p gpurun_out

timeout -k 10 500 python tools/variants.py run --only s0 c044 base --gib 64 --reps 16 > gpurun_out/bd_variants.json 2>gpurun_out/bd_variants.err
rc=$?
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/bd_variants.json"))
    print({k: v for k, v in d["agree"].items() if not v})
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
