#!/bin/bash
# new split-path tests (with the split-counter hook), then the whole GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "overflow_fallback or max_length" -v -p no:cacheprovider --timeout 240 --timeout-method thread -x > $O/r02ad_new.log 2>&1 || { tail -30 $O/r02ad_new.log; exit 1; }
tail -4 $O/r02ad_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02ad_tests.log 2>&1
rc=$?; tail -2 $O/r02ad_tests.log; exit $rc
