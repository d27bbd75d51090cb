#!/bin/bash
# fixed kernel: per-wave runs + one coalesced result store per run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/p_tests.log 2>&1 && \
timeout -k 10 300 python tools/variants.py run --only base v3 --gib 64 --reps 7 > gpurun_out/p_variants.json 2>gpurun_out/p_variants.err
rc=$?
tail -3 gpurun_out/p_tests.log
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/p_variants.json"))
    print(d["agree"])
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
