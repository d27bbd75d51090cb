#!/bin/bash
# Probe: fixed kernel pair folded as one dependent chain (chain) vs two chains (base), far_pair for scale
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base chain far_pair --gib 64 --reps 7 > $O/s3b_variants.json 2> $O/s3b_variants.err || { tail -20 $O/s3b_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3b_variants.json"))
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
