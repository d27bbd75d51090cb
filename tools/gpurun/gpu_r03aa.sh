#!/bin/bash
# A/B: one-launch ring fold with unconditional per-stream head feeds and realignments vs HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03aa_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03aa_new.log; exit 1; }
tail -2 $O/r03aa_new.log
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 8 --only base prev --work file_desc file_verify tiny_desc adversarial > $O/r03aa_variants.json 2> $O/r03aa_variants.err || { tail -20 $O/r03aa_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03aa_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
timeout -k 10 300 python -u tools/percall.py > $O/r03aa_percall.json 2> $O/r03aa_percall.err || { tail -20 $O/r03aa_percall.err; exit 1; }
cat $O/r03aa_percall.json
