#!/bin/bash
# where the one-launch kernel's wave cycles go per SST file: active VALU / scalar / LDS instruction cycles, waits
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/cyc; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-include-regex crc32c_direct_kernel --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d $O/a -o run --output-format csv -- python3 $R/tools/run_file.py 5 > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-include-regex crc32c_direct_kernel --pmc SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -d $O/b -o run --output-format csv -- python3 $R/tools/run_file.py 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python3 $R/tools/pmc_per_unit.py $O crc32c_direct_kernel 16812 --label cycles_per_span
