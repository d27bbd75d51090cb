#!/bin/bash
# A/B quad kernel ring depth 2 vs 3 (and v2 as committed)
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only quadv2 quad_r2 quad_r3 --gib 16 --reps 10 > $O/r02i_variants.json 2> $O/r02i_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02i_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
