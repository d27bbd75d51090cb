#!/bin/bash
# A/B: sealing lane kernel touching the header line with the record's last task
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/variants.py run --gib 16 --reps 8 --only base lane_seal_touch --work wal wal_seal > $O/r03ac_variants.json 2> $O/r03ac_variants.err || { tail -20 $O/r03ac_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03ac_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(d['agree'])"
