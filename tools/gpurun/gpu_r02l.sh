#!/bin/bash
R=$(pwd); O=$R/gpurun_out/r02l; mkdir -p $O; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/run_quad_all.py > $O/kt.log 2>&1 || exit $?
cd $R && python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r02l/kt/run_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
for r in rows:
    if 'crc32c' in r['Kernel_Name'] or 'rocclr' in r['Kernel_Name']:
        print(f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:9.1f} us  {r['Kernel_Name'][:70]}")
PY
