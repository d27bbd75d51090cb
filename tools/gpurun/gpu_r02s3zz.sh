#!/bin/bash
# Session-3 close: GPU suite, smoke, default bench, secondary workloads on HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3zz_tests.log 2>&1 || { tail -20 $O/s3zz_tests.log; exit 1; }
tail -1 $O/s3zz_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3zz_smoke.log 2>&1 || { tail -20 $O/s3zz_smoke.log; exit 1; }
tail -1 $O/s3zz_smoke.log
timeout -k 10 600 python bench.py > $O/s3zz_bench.json 2> $O/s3zz_bench.err || exit $?
cat $O/s3zz_bench.json
