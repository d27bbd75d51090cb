#!/bin/bash
# host pipeline v2 (copy/compute streams, 32 MiB x 4, parallel staging): parity + e2e rate + copy timeline
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "host" --timeout 600 --timeout-method thread > gpurun_out/y_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --e2e --steps 1 --warmup 0 --nblocks 65536 --no-cpu-baseline > gpurun_out/y_e2e.json 2>gpurun_out/y_e2e.err && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/y_prof -o run --output-format csv -- python3 $R/bench.py --e2e --steps 1 --warmup 0 --nblocks 65536 --no-cpu-baseline > $R/gpurun_out/y_prof.log 2>&1
rc=$?
cd $R
tail -3 gpurun_out/y_tests.log
python -c "import json; d=json.loads(open('gpurun_out/y_e2e.json').read()); print(d.get('e2e_host_resident'))"
exit $rc
