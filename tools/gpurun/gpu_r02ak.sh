#!/bin/bash
# quad kernel with unaligned body loads (no head bytes): parity of the quad tests with that build, then the A/B
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/variants.py run --only quad_unaligned base --gib 16 --reps 10 > $O/r02ak_variants.json 2> $O/r02ak_variants.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02ak_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
