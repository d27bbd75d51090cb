#!/bin/bash
# launch floor probe + its kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/launch_floor.py > $O/r02ab_floor.json 2> $O/r02ab_floor.err || exit $?
cat $O/r02ab_floor.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r02ab_kt -o run --output-format csv -- python3 $R/tools/launch_floor.py > $O/r02ab_kt.log 2>&1
