#!/bin/bash
# span-kernel scalar bookkeeping probes (measurement-only variants)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/variants.py run --only base noswitch nonop noswitch_nonop --gib 64 --reps 7 > gpurun_out/am_variants.json 2>gpurun_out/am_variants.err
rc=$?
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/am_variants.json"))
    print(d["agree"])
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
