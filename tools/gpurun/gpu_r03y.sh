#!/bin/bash
# idle groups join ticket work on the help flag: direct tests, long-span batches and per-call vs HEAD, kernel trace of the per-call tool
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03y_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03y_new.log; exit 1; }
tail -2 $O/r03y_new.log
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 5 --only base prev --work huge64m adversarial file_desc file_verify tiny_desc > $O/r03y_variants.json 2> $O/r03y_variants.err || { tail -20 $O/r03y_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03y_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03y_kt -o run --output-format csv -- python3 $R/tools/percall.py > $O/r03y_percall_under_rocprof.json 2> $O/r03y_kt.log
cat $O/r03y_percall_under_rocprof.json
