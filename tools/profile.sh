#!/bin/bash
# rocprofv3 passes over the headline bench (run on the GPU box): kernel trace +
# stats of the default bench, then FETCH_SIZE, WRITE_SIZE and SQ/GRBM counters
# of the fixed kernel, each in a pass of its own (no --pmc together with any
# trace domain).  Output under $O/${TAG}_prof_*; summarise with
#   python tools/pmc_summary.py gpurun_out/<TAG> <TAG>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
B="python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-config5 --no-multi"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-multi > $O/prof_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex crc32c_fixed --pmc FETCH_SIZE -d $O/prof_fetch -o run --output-format csv -- $B > $O/prof_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex crc32c_fixed --pmc WRITE_SIZE -d $O/prof_write -o run --output-format csv -- $B > $O/prof_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex crc32c_fixed --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/prof_sq -o run --output-format csv -- $B > $O/prof_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex crc32c_fixed --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/prof_sq2 -o run --output-format csv -- $B > $O/prof_sq2.log 2>&1
