#!/bin/bash
# A/B: one-launch table fill retired after slot 0's first task
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 8 --only base tables_after_st0 --work file_desc file_verify tiny_desc huge64m adversarial > $O/r03z_variants.json 2> $O/r03z_variants.err || { tail -20 $O/r03z_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03z_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(d['agree'])"
