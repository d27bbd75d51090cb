#!/bin/bash
# one-launch kernel: table words at entry, ticket path in fewer round trips, stop-event launch, PRISMDB_CRC32C_UNORDERED:
# direct tests, per-call (ordered and unordered), A/B against the previous commit's kernel, timeline
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03q_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03q_new.log; exit 1; }
tail -2 $O/r03q_new.log
timeout -k 10 300 python -u tools/percall.py > $O/r03q_percall.json 2> $O/r03q_percall.err || { tail -20 $O/r03q_percall.err; exit 1; }
cat $O/r03q_percall.json
timeout -k 10 300 python -u tools/variants.py run --gib 8 --reps 8 --only base prev --work file_fixed file_desc file_verify tiny_desc sst3988 mixed > $O/r03q_variants.json 2> $O/r03q_variants.err || { tail -20 $O/r03q_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03q_variants.json'))
for w,r in d['results'].items(): print(w, {n: v['ms_median'] for n,v in r.items()})
print(all(d['agree'].values()))"
timeout -k 10 120 python -u tools/direct_timeline.py > $O/r03q_timeline.json 2> $O/r03q_timeline.err || { tail -20 $O/r03q_timeline.err; exit 1; }
timeout -k 10 120 python -u tools/direct_timeline.py --data-only >> $O/r03q_timeline.json 2>> $O/r03q_timeline.err || { tail -20 $O/r03q_timeline.err; exit 1; }
cat $O/r03q_timeline.json
