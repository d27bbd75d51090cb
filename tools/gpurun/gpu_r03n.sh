#!/bin/bash
# one-launch kernel: table fill order, ticket size, worker count (A/B) + timelines
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/variants.py run --gib 8 --reps 6 --only base tables_first lg0 workers2x tf_lg0_w2 --work file_fixed file_desc file_verify tiny_desc sst3988 > $O/r03n_variants.json 2> $O/r03n_variants.err || { tail -20 $O/r03n_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03n_variants.json'))
for w,r in d['results'].items(): print(w, {n: v['ms_median'] for n,v in r.items()})
print(all(d['agree'].values()))"
for v in direct_ts tf_ts; do
timeout -k 10 120 python -u tools/direct_timeline.py --lib tools/_build/variants/lib_$v.so > $O/r03n_timeline_$v.json 2> $O/r03n_timeline.err || { tail -20 $O/r03n_timeline.err; exit 1; }
cat $O/r03n_timeline_$v.json
done
