#!/bin/bash
# PMC passes over the WAL verify workload (tools/run_wal.py): quad kernel and
# the rest of the launch sequence.  One counter group per pass (no --pmc with
# any trace domain); run on the GPU box from the repo root.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-quad}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp || exit 1
K=${2:-crc32c_quad_kernel}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/run_wal.py 3 > $O/kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/sq -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/sq2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR -d $O/sq3 -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/sq3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/fetch.log 2>&1
