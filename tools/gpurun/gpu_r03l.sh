#!/bin/bash
# burst probe (file-sized call floor), full GPU suite on the early-issue kernel, per-call trace, WAL lane kernel seal vs verify PMC (FETCH_SIZE / WRITE_SIZE, own passes)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
for b in 67529245 268435456 16777216; do timeout -k 10 120 $R/tools/_build/burstprobe $b >> $O/r03l_burst.json 2>&1 || { cat $O/r03l_burst.json; exit 1; }; done
cat $O/r03l_burst.json
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03l_smoke.log 2>&1 || { tail -20 $O/r03l_smoke.log; exit 1; }
tail -1 $O/r03l_smoke.log
timeout -k 10 800 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03l_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03l_tests.log; exit 1; }
tail -2 $O/r03l_tests.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03l_kt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r03l_percall_under_rocprof.json 2> $O/r03l_kt.log || { tail -5 $O/r03l_kt.log; exit 1; }
cat $O/r03l_percall_under_rocprof.json
timeout -s KILL 300 rocprofv3 --kernel-include-regex crc32c_lane --pmc FETCH_SIZE -d $O/r03l_wal_fetch -o run --output-format csv -- python3 $R/tools/bench_configs.py --only wal --reps 2 > $O/r03l_wal_fetch.log 2>&1 || { tail -5 $O/r03l_wal_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex crc32c_lane --pmc WRITE_SIZE -d $O/r03l_wal_write -o run --output-format csv -- python3 $R/tools/bench_configs.py --only wal --reps 2 > $O/r03l_wal_write.log 2>&1 || { tail -5 $O/r03l_wal_write.log; exit 1; }
grep -h "wal_" -A 6 $O/r03l_wal_write.log | head -30
