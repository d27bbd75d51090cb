#!/bin/bash
# A/B: HEAD vs the kernel source before pair runs (commit 1c4162b): general-kernel register changes
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only older_src base --gib 16 --reps 10 > $O/r02al_variants.json 2> $O/r02al_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02al_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
