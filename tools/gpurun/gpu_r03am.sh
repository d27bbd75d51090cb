#!/bin/bash
# A/B: one-launch edge bytes packed per quad by DPP (fewer readlanes and scalar shifts per span) vs HEAD; direct tests first
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py tests/test_log.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/r03am_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03am_new.log; exit 1; }
tail -2 $O/r03am_new.log
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 10 --only base prev --work file_desc file_verify tiny_desc adversarial > $O/r03am_variants.json 2> $O/r03am_variants.err || { tail -20 $O/r03am_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03am_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
timeout -k 10 400 bash $R/tools/gpurun/gpu_r03an.sh > $O/r03an.log 2>&1 || { echo AN_FAIL; tail -20 $O/r03an.log; exit 1; }
cat $O/r03an.log
