#!/bin/bash
# Round 3: one-launch descriptor path -- smoke, its tests, the full GPU suite, per-call cost
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03b_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/r03b_smoke.log; exit 1; }
tail -2 $O/r03b_smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/r03b_direct.log 2>&1 || { echo DIRECT_FAIL; tail -40 $O/r03b_direct.log; exit 1; }
tail -3 $O/r03b_direct.log
timeout -k 10 300 python -u tools/percall.py > $O/r03b_percall.json 2> $O/r03b_percall.err || { echo PERCALL_FAIL; tail -20 $O/r03b_percall.err; exit 1; }
cat $O/r03b_percall.json
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03b_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03b_tests.log; exit 1; }
tail -3 $O/r03b_tests.log
