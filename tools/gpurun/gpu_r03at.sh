#!/bin/bash
# planner path: SST-shaped descriptors plain vs sealed (trailer stores in the span kernel's ring)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 6 --only base --work sst3988 sst3988_seal > $O/r03at_variants.json 2> $O/r03at_variants.err || { tail -20 $O/r03at_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03at_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})"
