#!/bin/bash
# Lane kernel v3: load-pattern ceiling (no fold), PMC profile, secondary workloads
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 600 python tools/variants.py run --only base lane_nofold --work wal --gib 32 --reps 5 > $O/s3j_variants.json 2> $O/s3j_variants.err || { tail -20 $O/s3j_variants.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3j_variants.json"))
for w, r in d["results"].items():
    print(w, {n: v["GB/s_median"] for n, v in r.items()})
PY
bash tools/prof_quad.sh s3j_lane crc32c_lane_kernel || exit $?
cd $R
timeout -k 10 600 python tools/bench_configs.py > $O/s3j_configs.json 2> $O/s3j_configs.err || { tail -20 $O/s3j_configs.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3j_configs.json"))
for w, r in d["results"].items():
    print(w, {k: v for k, v in r.items() if k in ("GiB/s", "roofline_frac", "mismatches")})
PY
