#!/bin/bash
# runs + coalesced nt result stores in both kernels: parity, stress, A/B vs v3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/q_tests.log 2>&1 && \
timeout -k 10 300 python tools/debug_span2.py > gpurun_out/q_stress.log 2>&1 && \
timeout -k 10 300 python tools/variants.py run --only base v3 --gib 64 --reps 7 > gpurun_out/q_variants.json 2>gpurun_out/q_variants.err
rc=$?
tail -3 gpurun_out/q_tests.log; grep -c "mismatches=0" gpurun_out/q_stress.log
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/q_variants.json"))
    print(d["agree"])
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
PY
exit $rc
