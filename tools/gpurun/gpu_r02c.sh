#!/bin/bash
# Kernel trace of the secondary workloads: where config 3 / sst_desc / WAL time goes per kernel.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/r02c_kt -o run --output-format csv -- python3 $R/tools/bench_configs.py --reps 3 > $O/r02c_configs.json 2> $O/r02c_configs.err || exit $?
find $O/r02c_kt -name '*.csv' | head
