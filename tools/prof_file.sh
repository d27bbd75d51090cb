#!/bin/bash
# PMC passes for the one-launch kernel at the per-file granularity (tools/run_file.py):
# instruction mix and wave cycles, then HBM bytes (FETCH_SIZE, WRITE_SIZE) in passes of their own.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pf; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
K=crc32c_direct_kernel
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/run_file.py 20 > $O/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/sq -o run --output-format csv -- python3 $R/tools/run_file.py 5 > $O/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/tools/run_file.py 5 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/tools/run_file.py 5 > $O/write.log 2>&1 || exit $?
echo prof_file done
