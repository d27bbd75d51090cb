#!/bin/bash
# Lane kernel with 8 waves (base) vs s_setprio 3 around the line loads (8 and 12 waves) per CU
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base lane_prio3 lane_w12_prio3 --work wal wal_seal --gib 32 --reps 7 > $O/s3t_variants.json 2> $O/s3t_variants.err || { tail -20 $O/s3t_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3t_variants.json"))
print({k: v for k, v in d["agree"].items() if not v})
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
