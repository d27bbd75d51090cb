#!/bin/bash
# engine + gather with two ranks on the device; PMC passes of the one-launch kernel per SST file
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/r03ad_dist.log 2>&1 || { echo DIST_FAIL; tail -60 $O/r03ad_dist.log; exit 1; }
tail -3 $O/r03ad_dist.log
timeout -k 10 600 bash $R/tools/prof_file.sh > $O/r03ad_prof.log 2>&1 || { echo PROF_FAIL; tail -30 $O/r03ad_prof.log; exit 1; }
cat $O/r03ad_prof.log
python3 $R/tools/pmc_per_unit.py $O/pf crc32c_direct_kernel 16812 --label per_span > $O/r03ad_pmc_per_span.json && cat $O/r03ad_pmc_per_span.json
