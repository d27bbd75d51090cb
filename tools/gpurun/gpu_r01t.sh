#!/bin/bash
# power/clock samples while the fixed kernel (base vs nofold) runs back to back
set -o pipefail
mkdir -p gpurun_out
rocm-smi --showpower --showclocks --showtemp --showmaxpower --json > gpurun_out/t_idle.json 2>&1
timeout -k 10 200 python tools/power_probe.py --only base nofold base nofold --seconds 6 > gpurun_out/t_power.log 2>&1
rc=$?
cat gpurun_out/t_power.log | tail -6
head -c 1500 gpurun_out/t_idle.json
exit $rc
