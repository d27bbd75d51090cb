#!/bin/bash
# the hardware floor of a file-sized call: empty launch, LDS fill, 67 MB streaming read (tools/burstprobe.hip)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 120 $R/tools/_build/burstprobe > $O/r03k_burst.json 2>&1 || { cat $O/r03k_burst.json; exit 1; }
timeout -k 10 120 $R/tools/_build/burstprobe 268435456 >> $O/r03k_burst.json 2>&1 || { cat $O/r03k_burst.json; exit 1; }
timeout -k 10 120 $R/tools/_build/burstprobe 16777216 >> $O/r03k_burst.json 2>&1 || { cat $O/r03k_burst.json; exit 1; }
cat $O/r03k_burst.json
