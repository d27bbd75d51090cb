#!/bin/bash
# ring up to 32 chunks, tickets >= 4 chunks, pipelined ticket folds: GPU suite, per-call, long-span batches vs HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03x_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03x_new.log; exit 1; }
tail -2 $O/r03x_new.log
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03x_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03x_tests.log; exit 1; }
tail -2 $O/r03x_tests.log
timeout -k 10 300 python -u tools/percall.py > $O/r03x_percall.json 2> $O/r03x_percall.err || { tail -20 $O/r03x_percall.err; exit 1; }
cat $O/r03x_percall.json
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 5 --only base prev --work huge64m adversarial file_desc file_verify tiny_desc > $O/r03x_variants.json 2> $O/r03x_variants.err || { tail -20 $O/r03x_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03x_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
