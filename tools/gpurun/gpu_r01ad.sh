#!/bin/bash
# kernel-trace breakdown of the generic path on 16 Mi x 4 KiB descriptors (plan / slice scan / mark / span)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ad_kt -o run --output-format csv -- python3 $R/tools/run_desc4k.py 5 > $O/ad_kt.log 2>&1
rc=$?
cat $O/ad_kt/*/run_kernel_stats.csv 2>/dev/null | cut -c1-200 || find $O/ad_kt -name "*stats*"
exit $rc
