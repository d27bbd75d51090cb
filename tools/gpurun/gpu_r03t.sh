#!/bin/bash
# one-launch kernel: ring-folded spans of up to 16 chunks, tagged hand-offs: full GPU suite, per-call, chunked probe, A/B vs HEAD, WAL seal store probe
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03t_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03t_new.log; exit 1; }
tail -2 $O/r03t_new.log
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03t_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/r03t_tests.log; exit 1; }
tail -2 $O/r03t_tests.log
timeout -k 10 300 python -u tools/percall.py > $O/r03t_percall.json 2> $O/r03t_percall.err || { tail -20 $O/r03t_percall.err; exit 1; }
cat $O/r03t_percall.json
timeout -k 10 300 python -u tools/chunked_direct.py > $O/r03t_chunked.json 2> $O/r03t_chunked.err || { tail -20 $O/r03t_chunked.err; exit 1; }
cat $O/r03t_chunked.json
timeout -k 10 400 python -u tools/variants.py run --gib 16 --reps 8 --only base prev lane_noseal --work file_desc file_verify tiny_desc sst3988 mixed wal wal_seal > $O/r03t_variants.json 2> $O/r03t_variants.err || { tail -20 $O/r03t_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03t_variants.json'))
for w,r in d['results'].items(): print(w, {n: v['ms_median'] for n,v in r.items()})
print(d['agree'])"
