#!/bin/bash
# GPU call: parity tests, bandwidth probes vs engine kernels, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; ok $rc || exit $rc
timeout -k 10 600 python tools/bwprobe.py --gib 16 --reps 5 > gpurun_out/bwprobe.json 2> gpurun_out/bwprobe.err
rc=$?; ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
