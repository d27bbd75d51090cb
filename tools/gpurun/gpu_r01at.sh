#!/bin/bash
# GPU parity suite at HEAD (+ small-pad immediate-offset loads)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/at_tests.log 2>&1
rc=$?
tail -2 gpurun_out/at_tests.log
grep -E "FAILED|Error" gpurun_out/at_tests.log | head -10
exit $rc
