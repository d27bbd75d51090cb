#!/bin/bash
# GPU call: variant sweep + rocprofv3 kernel trace + PMC passes on the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python tools/variants.py run --gib 64 --reps 7 > gpurun_out/variants.json 2> gpurun_out/variants.err
rc=$?; ok $rc || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_kt.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 600 rocprofv3 --kernel-include-regex crc32c_fixed --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof_fetch.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 600 rocprofv3 --kernel-include-regex crc32c_fixed --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof_write.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 600 rocprofv3 --kernel-include-regex crc32c_fixed --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/prof_sq -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof_sq.log 2>&1
rc=$?; ok $rc || exit $rc
timeout -k 10 600 rocprofv3 --kernel-include-regex crc32c_fixed --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d $R/gpurun_out/prof_sq2 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof_sq2.log 2>&1
