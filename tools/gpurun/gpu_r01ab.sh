#!/bin/bash
# span-kernel round-skip ceiling: rounds >= 12 only / no rounds (measurement-only, wrong results)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/variants.py run --only base span_j12 span_j16 --gib 64 --reps 7 > gpurun_out/ab_variants.json 2>gpurun_out/ab_variants.err
rc=$?
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/ab_variants.json"))
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
