#!/bin/bash
# Lane kernel fuzz campaign: 60 seeds of the randomized suite (all three routing modes)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PRISMDB_FUZZ_SEEDS=60 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/s3y_fuzz.log 2>&1 || { tail -30 $O/s3y_fuzz.log; exit 1; }
tail -2 $O/s3y_fuzz.log
