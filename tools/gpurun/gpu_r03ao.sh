#!/bin/bash
# 60-seed fuzz campaign on the final build (all routes), then the direct tests again
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
export PRISMDB_FUZZ_SEEDS=60
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 300 --timeout-method thread -m gpu > $O/r03ao_fuzz.log 2>&1 || { echo FUZZ_FAIL; tail -60 $O/r03ao_fuzz.log; exit 1; }
tail -2 $O/r03ao_fuzz.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py -q --timeout 200 --timeout-method thread -m gpu -k random_batches > $O/r03ao_random.log 2>&1 || { echo RANDOM_FAIL; tail -60 $O/r03ao_random.log; exit 1; }
tail -2 $O/r03ao_random.log
