#!/bin/bash
# A/B: span-kernel slices per stream 16 (base) / 64 / 256: tail balance of the static slice schedule
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only base slices64 slices256 --gib 16 --reps 10 > $O/r02p_variants.json 2> $O/r02p_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02p_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
