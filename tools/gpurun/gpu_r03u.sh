#!/bin/bash
# one-launch ring chunk index packed in the task flags; lane-kernel seal stores moved to crc32c_lane_seal_kernel: direct/log/parity tests, per-call, A/B vs HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_direct.py tests/test_log.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03u_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03u_new.log; exit 1; }
tail -2 $O/r03u_new.log
timeout -k 10 300 python -u tools/percall.py > $O/r03u_percall.json 2> $O/r03u_percall.err || { tail -20 $O/r03u_percall.err; exit 1; }
cat $O/r03u_percall.json
timeout -k 10 400 python -u tools/variants.py run --gib 16 --reps 8 --only base prev --work file_desc file_verify tiny_desc wal wal_seal > $O/r03u_variants.json 2> $O/r03u_variants.err || { tail -20 $O/r03u_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03u_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
timeout -k 10 400 python -u tools/bench_configs.py --only wal_seal wal_verify config3_mixed sst_desc > $O/r03u_configs.json 2> $O/r03u_configs.err || { tail -20 $O/r03u_configs.err; exit 1; }
cat $O/r03u_configs.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r03u_kt -o run --output-format csv -- python3 $R/tools/bench_configs.py --reps 3 --only sst_desc config3_mixed > $O/r03u_configs_under_rocprof.json 2> $O/r03u_kt.log
