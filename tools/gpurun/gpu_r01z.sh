#!/bin/bash
# bisect the exit-time crash seen under rocprofv3 --memory-copy-trace with the new host pipeline
mkdir -p gpurun_out
R=$(pwd)
export TMPDIR=/tmp
cd /tmp
PRISMDB_STAGE_THREADS=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/z1 -o run --output-format csv -- python3 $R/bench.py --e2e --steps 1 --warmup 0 --nblocks 65536 --no-cpu-baseline > $R/gpurun_out/z1.log 2>&1
echo "threads=1 memcpy-trace rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/z2 -o run --output-format csv -- python3 $R/bench.py --e2e --steps 1 --warmup 0 --nblocks 65536 --no-cpu-baseline > $R/gpurun_out/z2.log 2>&1
echo "kernel-trace only rc=$?"
exit 0
