#!/bin/bash
# fuzz campaign: 60 seeds of every randomized test (pair batches included), once
set -o pipefail
O=gpurun_out; mkdir -p $O
export PRISMDB_FUZZ_SEEDS=60
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02am_fuzz.log 2>&1
rc=$?; tail -3 $O/r02am_fuzz.log; exit $rc
