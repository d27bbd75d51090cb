#!/bin/bash
# Round-2 session-3 re-entry check: GPU suite, smoke, default bench, bench under rocprofv3 --kernel-trace --stats
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3_tests.log 2>&1 || { tail -20 $O/s3_tests.log; exit 1; }
tail -1 $O/s3_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3_smoke.log 2>&1 || { tail -20 $O/s3_smoke.log; exit 1; }
tail -2 $O/s3_smoke.log
timeout -k 10 600 python bench.py > $O/s3_bench.json 2> $O/s3_bench.err || exit $?
cat $O/s3_bench.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/s3_kt -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/s3_bench_under_rocprof.json 2> $O/s3_kt.log || exit $?
cat $O/s3_bench_under_rocprof.json
grep -h "crc32c_fixed" $O/s3_kt/run_kernel_stats.csv
