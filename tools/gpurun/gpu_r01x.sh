#!/bin/bash
# host-resident pipeline timeline: kernel + memory-copy trace of bench --e2e
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --e2e --steps 1 --warmup 0 --nblocks 65536 --no-cpu-baseline > gpurun_out/x_e2e.json 2>gpurun_out/x_e2e.err && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/x_prof -o run --output-format csv -- python3 $R/bench.py --e2e --steps 1 --warmup 0 --nblocks 65536 --no-cpu-baseline > $R/gpurun_out/x_prof.log 2>&1
rc=$?
cd $R
cat gpurun_out/x_e2e.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('e2e_host_resident'))"
ls gpurun_out/x_prof
exit $rc
