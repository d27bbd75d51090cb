#!/bin/bash
# one-launch kernel with tagged-word hand-offs (no release/acquire fences): direct tests, per-call, A/B against HEAD's kernel, timeline
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/r03s_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03s_new.log; exit 1; }
tail -2 $O/r03s_new.log
timeout -k 10 300 python -u tools/percall.py > $O/r03s_percall.json 2> $O/r03s_percall.err || { tail -20 $O/r03s_percall.err; exit 1; }
cat $O/r03s_percall.json
timeout -k 10 300 python -u tools/variants.py run --gib 8 --reps 8 --only base prev --work file_fixed file_desc file_verify tiny_desc sst3988 mixed > $O/r03s_variants.json 2> $O/r03s_variants.err || { tail -20 $O/r03s_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03s_variants.json'))
for w,r in d['results'].items(): print(w, {n: v['ms_median'] for n,v in r.items()})
print(all(d['agree'].values()))"
timeout -k 10 120 python -u tools/direct_timeline.py > $O/r03s_timeline.json 2> $O/r03s_timeline.err || { tail -20 $O/r03s_timeline.err; exit 1; }
timeout -k 10 120 python -u tools/direct_timeline.py --data-only >> $O/r03s_timeline.json 2>> $O/r03s_timeline.err || { tail -20 $O/r03s_timeline.err; exit 1; }
cat $O/r03s_timeline.json
timeout -k 10 300 python -u tools/chunked_direct.py > $O/r03s_chunked.json 2> $O/r03s_chunked.err || { tail -20 $O/r03s_chunked.err; exit 1; }
cat $O/r03s_chunked.json
