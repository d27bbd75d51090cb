#!/bin/bash
# per-call times incl. distinct files; A/B span/fixed kernels at 16/12/8 waves per CU
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/percall.py > $O/r03ag_percall.json 2> $O/r03ag_percall.err || { tail -20 $O/r03ag_percall.err; exit 1; }
cat $O/r03ag_percall.json
timeout -k 10 600 python -u tools/variants.py run --gib 32 --reps 6 --only base waves12 waves8 --work sst3988 mixed fixed4k desc4k adversarial > $O/r03ag_variants.json 2> $O/r03ag_variants.err || { tail -20 $O/r03ag_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03ag_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(d['agree'])"
