#!/bin/bash
# log-record batching on the device + all secondary workloads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/i_tests.log 2>&1 && \
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/i_configs.json 2> gpurun_out/i_configs.err
rc=$?
tail -5 gpurun_out/i_tests.log; cat gpurun_out/i_configs.json; tail -3 gpurun_out/i_configs.err
exit $rc
