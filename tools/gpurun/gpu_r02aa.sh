#!/bin/bash
# A/B: planner segment records by the wave (base) vs one thread; span-kernel launch floor
# (return at entry / after the table load; measurement); GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only base plan_serial no_wg_exit --gib 16 --reps 10 > $O/r02aa_variants.json 2> $O/r02aa_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02aa_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: (v["GB/s_median"], v["ms_median"]) for n, v in r.items()})
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02aa_tests.log 2>&1
rc=$?; tail -2 $O/r02aa_tests.log; exit $rc
