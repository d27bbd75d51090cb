#!/bin/bash
# multi-threaded host callers test, then the whole suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k concurrent --timeout 200 --timeout-method thread > gpurun_out/bk_tests.log 2>&1 || { tail -20 gpurun_out/bk_tests.log; exit 1; }
tail -1 gpurun_out/bk_tests.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bk_all.log 2>&1 || { tail -5 gpurun_out/bk_all.log; exit 1; }
tail -1 gpurun_out/bk_all.log
