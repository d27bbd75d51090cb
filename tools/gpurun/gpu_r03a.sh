#!/bin/bash
# Round 3 baseline: per-call latency of one SST file's blocks + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/percall.py > $O/r03a_percall.json 2> $O/r03a_percall.err || exit $?
cat $O/r03a_percall.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03a_kt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r03a_kt.log 2>&1
