#!/bin/bash
# fixed-kernel issue sensitivity: +200 SALU or +64 VALU per span pair (measurement)
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only salu200 valu64 base --gib 16 --reps 10 > $O/r02y_variants.json 2> $O/r02y_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02y_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
