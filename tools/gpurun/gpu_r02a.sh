#!/bin/bash
# Round-2 baseline on a fresh box: headline bench line, secondary workloads.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py > $O/r02a_bench.json 2> $O/r02a_bench.err || exit $?
tail -1 $O/r02a_bench.json
timeout -k 10 400 python tools/bench_configs.py --reps 5 > $O/r02a_configs.json 2> $O/r02a_configs.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02a_configs.json"))
for k, v in d["results"].items():
    print(k, {x: v[x] for x in v if x in ("GiB/s", "roofline_frac", "GB/s")})
PY
