#!/bin/bash
# A/B: one-launch ring spans' trailers stored with the run's results after the ring vs HEAD; seal-covering tests first
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_direct.py tests/test_log.py tests/test_gpu_fuzz.py tests/test_sst.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/r03ar_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03ar_new.log; exit 1; }
tail -2 $O/r03ar_new.log
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 10 --only base prev --work file_seal file_desc file_verify tiny_desc > $O/r03ar_variants.json 2> $O/r03ar_variants.err || { tail -20 $O/r03ar_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03ar_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
