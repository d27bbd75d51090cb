#!/bin/bash
# one-launch path + batch_multi (ndev = 1): new tests first, full GPU suite, kernel trace of the per-call tool
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03g_smoke.log 2>&1 || { tail -20 $O/r03g_smoke.log; exit 1; }
tail -1 $O/r03g_smoke.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_multi.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/r03g_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03g_new.log; exit 1; }
tail -3 $O/r03g_new.log
timeout -k 10 800 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03g_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03g_tests.log; exit 1; }
tail -2 $O/r03g_tests.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03g_kt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r03g_percall_under_rocprof.json 2> $O/r03g_kt.log
