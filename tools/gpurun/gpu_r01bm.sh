#!/bin/bash
# log kernel: computed entry into the rounds + bfe masks: suite, A/B vs 44df566
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bm_tests.log 2>&1 || { tail -5 gpurun_out/bm_tests.log; exit 1; }
tail -1 gpurun_out/bm_tests.log
timeout -k 10 500 python tools/variants.py run --only prev base --gib 64 --reps 12 > gpurun_out/bm_variants.json 2>gpurun_out/bm_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/bm_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
