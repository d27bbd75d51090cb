#!/bin/bash
# A/B: per-file cost of the batch-size ticket sizing (base) vs the same without it (tlg64) vs HEAD (prev)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 10 --only base tlg64 prev --work file_desc file_verify tiny_desc > $O/r03ai_variants.json 2> $O/r03ai_variants.err || { tail -20 $O/r03ai_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03ai_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
