#!/bin/bash
# Session-3 final: GPU suite, smoke, default bench, bench under rocprofv3 --kernel-trace --stats,
# PMC passes on the headline kernel (tools/profile.sh), host-resident e2e rates
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3final_tests.log 2>&1 || { tail -20 $O/s3final_tests.log; exit 1; }
tail -1 $O/s3final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3final_smoke.log 2>&1 || { tail -20 $O/s3final_smoke.log; exit 1; }
tail -1 $O/s3final_smoke.log
timeout -k 10 600 python bench.py > $O/s3final_bench.json 2> $O/s3final_bench.err || exit $?
cat $O/s3final_bench.json
timeout -k 10 900 bash tools/profile.sh || exit $?
cd $R
python tools/pmc_summary.py $O r02s3final > $O/s3final_pmc.json 2> $O/s3final_pmc.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/s3final_pmc.json"))
print({k: d.get(k) for k in ("kernel_trace", "hbm_bytes_per_launch", "fetch_ratio", "hbm_GBps_from_pmc", "effective_clock_GHz")})
PY
grep -h "crc32c_fixed" $O/prof_kt/run_kernel_stats.csv
tail -1 $O/prof_kt.log
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 1 --no-cpu-baseline > $O/s3final_e2e.json 2> $O/s3final_e2e.err || exit $?
python - <<'PY'
import json
e = json.loads(open("gpurun_out/s3final_e2e.json").read().strip().splitlines()[-1])
print("e2e", e.get("e2e_host_resident"))
PY
