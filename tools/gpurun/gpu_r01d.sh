#!/bin/bash
# GPU call: parity tests, bench (+e2e), secondary workloads.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py --e2e > gpurun_out/bench.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.json 2> gpurun_out/configs.err
