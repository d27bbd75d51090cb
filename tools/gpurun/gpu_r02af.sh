#!/bin/bash
# measurement: fixed kernel pairing spans half a run apart
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only far_pair base --gib 16 --reps 10 > $O/r02af_variants.json 2> $O/r02af_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02af_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
