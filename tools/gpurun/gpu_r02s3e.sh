#!/bin/bash
# Lane kernel limits on WAL verify: loads only (nofold), 16-B aligned loads, the quad kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base lane_nofold lane_aligned quadk --work wal mixed --gib 32 --reps 5 > $O/s3e_variants.json 2> $O/s3e_variants.err || { tail -20 $O/s3e_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3e_variants.json"))
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
