#!/bin/bash
# LDS bank conflicts and LDS-array cycles of the one-launch kernel per SST file (vs the fixed kernel on the data blocks)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lds; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-include-regex crc32c_direct_kernel --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/direct -o run --output-format csv -- python3 $R/tools/run_file.py 5 > $O/direct.log 2>&1 || { tail -20 $O/direct.log; exit 1; }
python3 $R/tools/pmc_per_unit.py $O crc32c_direct_kernel 16812 --label lds_per_span
