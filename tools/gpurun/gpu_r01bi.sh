#!/bin/bash
# scan fused into the planner's last block, no slice kernels for n <= streams: suite, per-call, A/B vs 5437bc8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bi_tests.log 2>&1 || { tail -5 gpurun_out/bi_tests.log; exit 1; }
tail -1 gpurun_out/bi_tests.log
timeout -k 10 300 python tools/percall.py > gpurun_out/bi_percall.json 2> gpurun_out/bi_percall.err || exit $?
cat gpurun_out/bi_percall.json
timeout -k 10 500 python tools/variants.py run --only prev base --gib 64 --reps 12 > gpurun_out/bi_variants.json 2>gpurun_out/bi_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/bi_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
