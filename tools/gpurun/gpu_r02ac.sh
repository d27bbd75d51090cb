#!/bin/bash
# max-length span test first, then the whole GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "overflow_fallback or max_length" -v -p no:cacheprovider --timeout 240 --timeout-method thread -x > $O/r02ac_max.log 2>&1 || { tail -30 $O/r02ac_max.log; exit 1; }
tail -6 $O/r02ac_max.log
exit 0

