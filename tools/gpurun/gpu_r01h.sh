#!/bin/bash
# A/B v3 (base) vs v2 in one process, then the secondary workloads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/variants.py run --only base v2 --gib 64 --reps 7 > gpurun_out/h_variants.json 2>gpurun_out/h_variants.err && \
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/h_configs.json 2> gpurun_out/h_configs.err
rc=$?
cat gpurun_out/h_variants.json gpurun_out/h_configs.json
exit $rc
