#!/bin/bash
# per-wave phase timeline of the final one-launch kernel (one SST file; and data blocks only)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 120 python -u tools/direct_timeline.py > $O/r03ak_timeline.json 2> $O/r03ak_timeline.err || { tail -20 $O/r03ak_timeline.err; exit 1; }
timeout -k 10 120 python -u tools/direct_timeline.py --data-only >> $O/r03ak_timeline.json 2>> $O/r03ak_timeline.err || { tail -20 $O/r03ak_timeline.err; exit 1; }
cat $O/r03ak_timeline.json
