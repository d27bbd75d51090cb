#!/bin/bash
# Fixed kernel: pair loads issued at raised wave priority (s_setprio 1 / 3) vs base
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base setprio1 setprio3 --work fixed4k verify4k desc4k --gib 64 --reps 7 > $O/s3m_variants.json 2> $O/s3m_variants.err || { tail -20 $O/s3m_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3m_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
