#!/bin/bash
# Lane kernel with 8 (base) / 6 / 10 waves per CU
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base lane_w6 lane_w10 --work wal wal_seal --gib 32 --reps 7 > $O/s3q_variants.json 2> $O/s3q_variants.err || { tail -20 $O/s3q_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3q_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
