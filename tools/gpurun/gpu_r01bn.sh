#!/bin/bash
# GPU suite + smoke at HEAD (1b0c595)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bn_tests.log 2>&1 || { tail -5 gpurun_out/bn_tests.log; exit 1; }
tail -1 gpurun_out/bn_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
