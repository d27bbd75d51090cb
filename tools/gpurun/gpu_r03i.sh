#!/bin/bash
# host pipeline ring pool (threads) + where a file-sized one-launch call spends its time (variants)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "host_pipeline or host_batch" > $O/r03i_pipe.log 2>&1 || { echo PIPE_FAIL; tail -60 $O/r03i_pipe.log; exit 1; }
tail -3 $O/r03i_pipe.log
timeout -k 10 300 python -u tools/variants.py run --gib 8 --reps 6 --only base base2 direct_notables direct_nofold --work file_fixed file_desc file_verify tiny_desc > $O/r03i_variants.json 2> $O/r03i_variants.err || { tail -20 $O/r03i_variants.err; exit 1; }
cat $O/r03i_variants.json
