#!/bin/bash
# PMC instruction mix of the log-record span kernel (WAL verify, ~1 KB records) + GPU suite at HEAD
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/bl_tests.log 2>&1 || { tail -5 $O/bl_tests.log; exit 1; }
tail -1 $O/bl_tests.log
cd /tmp
K=crc32c_span_kernel
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/wl_kt -o run --output-format csv -- python3 $R/tools/run_wal.py 3 > $O/wl_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/wl_sq -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/wl_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/wl_sq2 -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/wl_sq2.log 2>&1 || exit $?
cd $R
python - <<'PY'
import csv, collections
n = None
for l in open("gpurun_out/wl_sq.log"):
    if l.startswith("records"):
        n = int(l.split()[1])
print("records", n)
for path in ["gpurun_out/wl_sq/run_counter_collection.csv", "gpurun_out/wl_sq2/run_counter_collection.csv"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "span_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in acc.items():
        print(c, round(max(d.values()) / n, 2), "per record (largest dispatch)")
PY
grep -i "crc32c" gpurun_out/wl_kt/run_kernel_stats.csv | cut -c1-150
