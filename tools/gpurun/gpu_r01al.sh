#!/bin/bash
# randomized parity (tests/test_gpu_fuzz.py) + the whole GPU suite, then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/al_tests.log 2>&1
rc=$?
tail -4 gpurun_out/al_tests.log
grep -E "FAILED|Error|assert" gpurun_out/al_tests.log | head -20
[ $rc -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/al_smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/al_smoke.log
exit $rc
