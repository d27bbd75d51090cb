#!/bin/bash
# max-length span test first, then the whole GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "max_length or huge_span or long_spans" -v -p no:cacheprovider --timeout 240 --timeout-method thread -x > $O/r02ac_max.log 2>&1 || { tail -30 $O/r02ac_max.log; exit 1; }
tail -6 $O/r02ac_max.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x --durations=5 > $O/r02ac_tests.log 2>&1
rc=$?; tail -9 $O/r02ac_tests.log; exit $rc
