#!/bin/bash
# re-entry validation of HEAD: gpu tests, smoke, default bench, rocprof kernel trace + PMC passes
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r_bench.json 2> gpurun_out/r_bench.err && \
bash tools/profile.sh && \
cd $R && python tools/pmc_summary.py gpurun_out r01r > gpurun_out/r_pmc.json
rc=$?
cd $R
tail -3 gpurun_out/r_tests.log; cat gpurun_out/r_smoke.log; cat gpurun_out/r_bench.json; tail -2 gpurun_out/r_bench.err
cat gpurun_out/r_pmc.json 2>/dev/null | head -40
exit $rc
