#!/bin/bash
# config-4 compaction leg (115 SST-shaped 64 MiB files, pageable, verify + seal through the host pipeline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --e2e --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ak_e2e.json 2> gpurun_out/ak_e2e.err
rc=$?
tail -3 gpurun_out/ak_e2e.err
python -c "
import json; d=json.loads(open('gpurun_out/ak_e2e.json').read().strip().splitlines()[-1]); print(json.dumps(d['e2e_host_resident']))"
exit $rc
