#!/bin/bash
# PMC instruction mix of both kernels after the xor3 change; torchrun N=1 launcher check
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
bash tools/profile.sh && bash tools/prof_desc.sh && cd $R && \
python tools/pmc_summary.py gpurun_out r01v > gpurun_out/v_pmc.json && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --nblocks 1048576 --no-cpu-baseline > gpurun_out/v_torchrun.log 2>&1
rc=$?
cd $R
tail -2 gpurun_out/v_torchrun.log
python - <<'PY'
import csv, collections
for name, path in [("fixed", "gpurun_out/prof_sq/run_counter_collection.csv"), ("span", "gpurun_out/pd_sq/run_counter_collection.csv"), ("span2", "gpurun_out/pd_sq2/run_counter_collection.csv"), ("fixed2", "gpurun_out/prof_sq2/run_counter_collection.csv")]:
    acc = collections.defaultdict(list)
    try:
        for r in csv.DictReader(open(path)):
            acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    except Exception as e:
        print(name, e); continue
    for k, v in sorted(acc.items()):
        print(name, k, round(sum(v) / len(v) / (1 << 24), 2), "per block")
PY
grep -i "crc32c" gpurun_out/pd_kt/run_kernel_stats.csv | cut -c1-160
exit $rc
