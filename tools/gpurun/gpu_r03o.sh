#!/bin/bash
# table-fill contention probe; one-launch path with the stop-event launch: direct tests + per-call
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 120 $R/tools/_build/burstprobe > $O/r03o_burst.json 2>&1 || { cat $O/r03o_burst.json; exit 1; }
cat $O/r03o_burst.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03o_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03o_new.log; exit 1; }
tail -2 $O/r03o_new.log
timeout -k 10 300 python -u tools/percall.py > $O/r03o_percall.json 2> $O/r03o_percall.err || { tail -20 $O/r03o_percall.err; exit 1; }
cat $O/r03o_percall.json
