#!/bin/bash
# Round-2 refresh at HEAD: bench line, rocprofv3 kernel trace + PMC passes, secondary workloads, host-resident e2e.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py > $O/r02n_bench.json 2> $O/r02n_bench.err || exit $?
tail -1 $O/r02n_bench.json
timeout -k 10 900 bash tools/profile.sh || exit $?
python tools/pmc_summary.py $O r02 > $O/r02n_pmc.json 2> $O/r02n_pmc.err || exit $?
timeout -k 10 400 python tools/bench_configs.py --reps 5 > $O/r02n_configs.json 2> $O/r02n_configs.err || exit $?
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 1 --no-cpu-baseline > $O/r02n_e2e.json 2> $O/r02n_e2e.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02n_configs.json"))
for k, v in d["results"].items():
    print(k, {x: v[x] for x in v if x in ("GiB/s", "roofline_frac", "ms")})
p = json.load(open("gpurun_out/r02n_pmc.json"))
print("pmc", p.get("hbm_bytes_per_launch"), p.get("fetch_ratio"), p.get("effective_clock_GHz"), p.get("instructions_per_block"))
e = json.loads(open("gpurun_out/r02n_e2e.json").read().strip().splitlines()[-1])
print("e2e", e.get("e2e_host_resident"))
PY
