#!/bin/bash
# SALU/VALU per WAL record for the shipped log kernel and two variants (PMC, kernel-filtered)
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
for v in base noskip inj0; do
  export PRISMDB_LIB=$R/tools/_build/variants/lib_$v.so
  timeout -k 10 300 rocprofv3 --kernel-include-regex crc32c_span_kernel --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/bp_$v -o run --output-format csv -- python3 $R/tools/run_wal.py 1 > $O/bp_$v.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bpk_$v -o run --output-format csv -- python3 $R/tools/run_wal.py 3 > $O/bpk_$v.log 2>&1 || exit $?
done
unset PRISMDB_LIB
cd $R
python - <<'PY'
import csv, collections
n = 4352000
for v in ["base", "noskip", "inj0"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f"gpurun_out/bp_{v}/run_counter_collection.csv")):
        if "span_kernel<true, true>" in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    row = {c: round(max(d.values()) / n, 1) for c, d in acc.items() if c.startswith("SQ_INSTS")}
    t = [l for l in open(f"gpurun_out/bpk_{v}/run_kernel_stats.csv") if "span_kernel<true, true>" in l]
    print(v, row, t[0].split(",")[3] if t else None)
PY
