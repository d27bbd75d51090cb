#!/bin/bash
# GPU suite + smoke after the ADVICE fixes (pipeline drain on failure, bounds checks, stream ordering).
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/r02b_tests.log 2>&1
rc=$?; tail -5 $O/r02b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r02b_smoke.log 2>&1 || exit $?
tail -2 $O/r02b_smoke.log
