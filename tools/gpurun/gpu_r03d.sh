#!/bin/bash
# per-call cost of one SST file (one-launch vs planner) + kernel trace of the same run
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/percall.py > $O/r03d_percall.json 2> $O/r03d_percall.err || { tail -20 $O/r03d_percall.err; exit 1; }
cat $O/r03d_percall.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03d_kt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r03d_kt.log 2>&1
