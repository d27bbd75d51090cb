#!/bin/bash
# round-3 PMC of the headline kernel (config 2): kernel trace, FETCH_SIZE, WRITE_SIZE, SQ passes; summary json for bench's roofline.traffic
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 1000 bash $R/tools/profile.sh > $O/r03aw_profile.log 2>&1 || { echo PROF_FAIL; tail -30 $O/r03aw_profile.log; exit 1; }
python3 $R/tools/pmc_summary.py $O r03aw > $O/r03aw_pmc.json && cat $O/r03aw_pmc.json
