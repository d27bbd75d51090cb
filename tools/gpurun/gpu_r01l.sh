#!/bin/bash
# read-pattern probes: grid-stride vs the CRC kernels' block pattern, 16 and 64 GiB buffers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bwprobe.py --gib 16 --reps 5 --blocks-only > gpurun_out/l_bw16.json 2>gpurun_out/l_bw16.err && \
timeout -k 10 300 python tools/bwprobe.py --gib 64 --reps 5 --blocks-only > gpurun_out/l_bw64.json 2>gpurun_out/l_bw64.err
rc=$?
python - <<'PY'
import json
for f in ("gpurun_out/l_bw16.json", "gpurun_out/l_bw64.json"):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(f, e); continue
    print(f)
    for k, v in d["results"].items():
        print(f"  {k:32s} {v['GB/s_median']:8.1f} best {v['GB/s_best']:8.1f}")
PY
exit $rc
