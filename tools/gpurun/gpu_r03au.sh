#!/bin/bash
# span kernel: trailers stored with the slice's results (flush) instead of from finish; seal-covering tests, A/B vs HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_sst.py tests/test_log.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/r03au_new.log 2>&1 || { echo NEW_FAIL; tail -60 $O/r03au_new.log; exit 1; }
tail -2 $O/r03au_new.log
timeout -k 10 400 python -u tools/variants.py run --gib 8 --reps 6 --only base prev --work sst3988_seal sst3988 mixed wal_seal > $O/r03au_variants.json 2> $O/r03au_variants.err || { tail -20 $O/r03au_variants.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r03au_variants.json'))
for w,r in d['results'].items(): print(w, {n: (v['ms_median'], v['GB/s_median']) for n,v in r.items()})
print(all(d['agree'].values()))"
