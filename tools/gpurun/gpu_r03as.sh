#!/bin/bash
# final-tree check: smoke, full GPU suite, bench (default), kernel trace of the bench, secondary workloads, per-call kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03as_smoke.log 2>&1 || { tail -20 $O/r03as_smoke.log; exit 1; }
tail -1 $O/r03as_smoke.log
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03as_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03as_tests.log; exit 1; }
tail -2 $O/r03as_tests.log
timeout -k 10 400 python -u bench.py > $O/r03as_bench.json 2> $O/r03as_bench.err || { tail -20 $O/r03as_bench.err; exit 1; }
cat $O/r03as_bench.json
timeout -k 10 400 python -u tools/bench_configs.py > $O/r03as_configs.json 2> $O/r03as_configs.err || { tail -20 $O/r03as_configs.err; exit 1; }
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r03as_kt -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 > $O/r03as_bench_under_rocprof.json 2> $O/r03as_kt.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03as_pkt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r03as_percall_under_rocprof.json 2> $O/r03as_pkt.log
