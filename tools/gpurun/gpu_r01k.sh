#!/bin/bash
# where does the fixed kernel's time go: with vs without the CRC fold
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/variants.py run --only base nofold nofold_nt0 --gib 64 --reps 7 > gpurun_out/k_variants.json 2>gpurun_out/k_variants.err
rc=$?
python - <<'PY'
import json
d = json.load(open("gpurun_out/k_variants.json"))
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
exit $rc
