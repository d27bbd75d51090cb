#!/bin/bash
# one-launch path (3 streams, 12 waves/CU, ticket workers): tests + per-call cost + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03f_smoke.log 2>&1 || { tail -20 $O/r03f_smoke.log; exit 1; }
tail -1 $O/r03f_smoke.log
timeout -k 10 300 python -u tools/percall.py > $O/r03f_percall.json 2> $O/r03f_percall.err || { tail -20 $O/r03f_percall.err; exit 1; }
cat $O/r03f_percall.json
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03f_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03f_tests.log; exit 1; }
tail -2 $O/r03f_tests.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03f_kt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r03f_percall_under_rocprof.json 2> $O/r03f_kt.log
