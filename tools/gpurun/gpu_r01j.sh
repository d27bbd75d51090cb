#!/bin/bash
# short-span path (lane-parallel head/tail, leading-round skip): parity, then A/B vs v3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/j_tests.log 2>&1 && \
timeout -k 10 300 python tools/debug_span2.py > gpurun_out/j_stress.log 2>&1 && \
timeout -k 10 400 python tools/variants.py run --only base v3 --gib 64 --reps 7 > gpurun_out/j_variants.json 2>gpurun_out/j_variants.err
rc=$?
tail -3 gpurun_out/j_tests.log; cat gpurun_out/j_stress.log gpurun_out/j_variants.json; tail -3 gpurun_out/j_variants.err
exit $rc
