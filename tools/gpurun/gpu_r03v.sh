#!/bin/bash
# one-launch path on batches with long spans (<= 2^17 spans): huge 64 MiB spans, adversarial lengths 0..70000, vs HEAD; planner route for reference
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 3 --only base prev --work huge64m adversarial mixed > $O/r03v_variants.json 2> $O/r03v_variants.err || { tail -20 $O/r03v_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03v_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(d['agree'])"
