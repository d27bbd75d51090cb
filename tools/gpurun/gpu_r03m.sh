#!/bin/bash
# per-call event cost (hipEventRecord vs hipExtLaunchKernel stop event vs none) and a per-wave timeline of a file-sized one-launch call
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/variants.py run --gib 8 --reps 6 --only base noevent extstop --work file_fixed file_desc file_verify tiny_desc > $O/r03m_variants.json 2> $O/r03m_variants.err || { tail -20 $O/r03m_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03m_variants.json'))
for w,r in d['results'].items(): print(w, {n: v['ms_median'] for n,v in r.items()})
print(d['agree'])"
timeout -k 10 120 python -u tools/direct_timeline.py > $O/r03m_timeline.json 2> $O/r03m_timeline.err || { tail -20 $O/r03m_timeline.err; exit 1; }
timeout -k 10 120 python -u tools/direct_timeline.py --data-only >> $O/r03m_timeline.json 2>> $O/r03m_timeline.err || { tail -20 $O/r03m_timeline.err; exit 1; }
cat $O/r03m_timeline.json
