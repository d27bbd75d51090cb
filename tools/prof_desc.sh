#!/bin/bash
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
K=crc32c_span_kernel
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pd_kt -o run --output-format csv -- python3 $R/tools/run_desc4k.py 3 > $O/pd_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pd_sq -o run --output-format csv -- python3 $R/tools/run_desc4k.py 1 > $O/pd_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/pd_sq2 -o run --output-format csv -- python3 $R/tools/run_desc4k.py 1 > $O/pd_sq2.log 2>&1
