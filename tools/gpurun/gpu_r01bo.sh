#!/bin/bash
# PC sampling probe (host_trap, beta) on the WAL driver: hot instructions of the log-record span kernel
R=$(pwd); O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $O/bo_list.log 2>&1
grep -i -A12 "pc.sampl\|PC Sampling" $O/bo_list.log | head -30
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-trace -d $O/bo_pcs -o run --output-format csv -- python3 $R/tools/run_wal.py 2 > $O/bo_pcs.log 2>&1
rc=$?
echo "pc sampling rc=$rc"
tail -5 $O/bo_pcs.log
ls -la $O/bo_pcs 2>/dev/null | head
exit 0
