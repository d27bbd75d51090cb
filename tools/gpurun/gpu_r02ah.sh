#!/bin/bash
# secondary workloads after pair runs + span-kernel PMC on 16 Mi x 4 KiB descriptors
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python tools/bench_configs.py --reps 5 > $O/r02ah_configs.json 2> $O/r02ah_configs.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02ah_configs.json"))
for k, v in d["results"].items():
    print(k, v["GiB/s"], v["roofline_frac"])
PY
bash tools/prof_desc.sh
