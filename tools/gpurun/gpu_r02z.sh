#!/bin/bash
# Per-call latency of one SST file's blocks, plus a kernel trace of the same run
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/percall.py > $O/r02z_percall.json 2> $O/r02z_percall.err || exit $?
cat $O/r02z_percall.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r02z_kt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r02z_kt.log 2>&1
