#!/bin/bash
# span kernel v3 (record-driven): parity, stress vs fixed kernel, A/B vs v2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/g_tests.log 2>&1 && \
timeout -k 10 300 python tools/debug_span2.py > gpurun_out/g_stress.log 2>&1 && \
timeout -k 10 300 python tools/variants.py run --only base v2 --gib 64 --reps 7 > gpurun_out/g_variants.json 2>gpurun_out/g_variants.err
rc=$?
tail -3 gpurun_out/g_tests.log; cat gpurun_out/g_stress.log; cat gpurun_out/g_variants.json
exit $rc
