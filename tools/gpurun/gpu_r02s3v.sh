#!/bin/bash
# Lane kernel with lane kernel: side loads every task (base) vs only where needed (measure-only), no fold per CU
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base lane_nodummy lane_nofold --work wal wal_seal --gib 32 --reps 7 > $O/s3v_variants.json 2> $O/s3v_variants.err || { tail -20 $O/s3v_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3v_variants.json"))
print(d["agree"])
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
