#!/bin/bash
# tickets per span scaled with the batch size (few huge spans): direct tests, A/B vs HEAD incl. one 1 GiB span, the planner for reference
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/r03ah_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03ah_new.log; exit 1; }
tail -2 $O/r03ah_new.log
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 5 --only base prev --work one_huge huge64m adversarial file_desc tiny_desc > $O/r03ah_variants.json 2> $O/r03ah_variants.err || { tail -20 $O/r03ah_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03ah_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
