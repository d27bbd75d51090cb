#!/bin/bash
# Final pass at HEAD: GPU suite + smoke, bench line, rocprofv3 kernel trace + PMC, secondary workloads, e2e + compaction
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/bf_tests.log 2>&1 || { tail -5 $O/bf_tests.log; exit 1; }
tail -1 $O/bf_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/bf_smoke.log 2>&1 || exit $?
tail -1 $O/bf_smoke.log
timeout -k 10 300 python bench.py > $O/bf_bench.json 2> $O/bf_bench.err || exit $?
tail -1 $O/bf_bench.json
timeout -k 10 900 bash tools/profile.sh || exit $?
python tools/pmc_summary.py $O r01final > $O/bf_pmc.json 2> $O/bf_pmc.err || exit $?
timeout -k 10 400 python tools/bench_configs.py --reps 5 > $O/bf_configs.json 2> $O/bf_configs.err || exit $?
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 1 --no-cpu-baseline > $O/bf_e2e.json 2> $O/bf_e2e.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/bf_configs.json"))
for k, v in d["results"].items():
    print(k, v["GiB/s"], v["roofline_frac"])
e = json.loads(open("gpurun_out/bf_e2e.json").read().strip().splitlines()[-1])
print("e2e", e.get("e2e_host_resident"))
PY
