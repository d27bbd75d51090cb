#!/bin/bash
# one-launch path: slot 0 issued before the table fill, no end-of-kernel counter, no idle-wave word reads: direct tests, then A/B (base = this tree, nodone = without the early issue, head = last commit)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_multi.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/r03j_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03j_new.log; exit 1; }
tail -3 $O/r03j_new.log
timeout -k 10 300 python -u tools/variants.py run --gib 8 --reps 6 --only base nodone head --work file_fixed file_desc file_verify tiny_desc sst3988 mixed > $O/r03j_variants.json 2> $O/r03j_variants.err || { tail -20 $O/r03j_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03j_variants.json'))
for w,r in d['results'].items(): print(w, {n: v['ms_median'] for n,v in r.items()})
print(d['agree'])"
