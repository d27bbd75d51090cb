#!/bin/bash
# Final round refresh at HEAD: bench line, rocprofv3 kernel trace + PMC, secondary workloads, e2e + compaction
# PMC passes (tools/profile.sh), secondary workloads, host-resident e2e.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py > $O/ai_bench.json 2> $O/ai_bench.err || exit $?
tail -1 $O/ai_bench.json
timeout -k 10 900 bash tools/profile.sh || exit $?
python tools/pmc_summary.py $O r01ay > $O/ai_pmc.json 2> $O/ai_pmc.err || exit $?
timeout -k 10 400 python tools/bench_configs.py --reps 5 > $O/ai_configs.json 2> $O/ai_configs.err || exit $?
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 1 --no-cpu-baseline > $O/ai_e2e.json 2> $O/ai_e2e.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/ay_configs.json"))
for k, v in d["results"].items():
    print(k, {x: v[x] for x in v if x in ("GiB/s", "roofline_frac", "GB/s")})
e = json.loads(open("gpurun_out/ay_e2e.json").read().strip().splitlines()[-1])
print("e2e", e.get("e2e_host_resident"))
PY
