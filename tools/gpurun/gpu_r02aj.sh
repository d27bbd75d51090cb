#!/bin/bash
# pair runs excluded after a segment-workspace overflow: the tests, then the GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pair_run or overflow_fallback" -v -p no:cacheprovider --timeout 240 --timeout-method thread -x > $O/r02aj_new.log 2>&1 || { tail -40 $O/r02aj_new.log; exit 1; }
tail -5 $O/r02aj_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02aj_tests.log 2>&1
rc=$?; tail -2 $O/r02aj_tests.log; exit $rc
