#!/bin/bash
# A/B of quad-kernel knobs (measurement cuts, realign grouping, quad for all batches)
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only base quad_norealign quad_nomask quad_ra2 quad_ra1 quad_all --gib 16 --reps 8 > $O/r02h_variants.json 2> $O/r02h_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02h_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
