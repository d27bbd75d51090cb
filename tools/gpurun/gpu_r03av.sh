#!/bin/bash
# sanity on the final in-tree library: smoke, one-launch and parity tests, a short bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03av_smoke.log 2>&1 || { tail -20 $O/r03av_smoke.log; exit 1; }
tail -1 $O/r03av_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_parity.py tests/test_sst.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03av_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03av_tests.log; exit 1; }
tail -2 $O/r03av_tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/r03av_bench.json 2> $O/r03av_bench.err || { tail -20 $O/r03av_bench.err; exit 1; }
cut -c1-400 $O/r03av_bench.json
