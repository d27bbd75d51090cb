#!/bin/bash
# pair-run span kernel: its parity tests, the A/B against the general kernel alone, the GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pair_run or full_runs or long_spans_close or full_size" -v -p no:cacheprovider --timeout 240 --timeout-method thread -x > $O/r02ag_new.log 2>&1 || { tail -40 $O/r02ag_new.log; exit 1; }
tail -12 $O/r02ag_new.log
timeout -k 10 600 python tools/variants.py run --only base no_pair_runs --gib 16 --reps 10 > $O/r02ag_variants.json 2> $O/r02ag_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02ag_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02ag_tests.log 2>&1
rc=$?; tail -2 $O/r02ag_tests.log; exit $rc
