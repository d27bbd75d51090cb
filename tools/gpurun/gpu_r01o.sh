#!/bin/bash
# store-pattern probes (64 GiB)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bwprobe.py --gib 64 --reps 5 --blocks-only > gpurun_out/o_bw64.json 2>gpurun_out/o_bw64.err
rc=$?
python - <<'PY'
import json
d = json.load(open("gpurun_out/o_bw64.json"))
for k, v in d["results"].items():
    if "store" in k or k.startswith("crc") or k.startswith("runs") or k in ("read_w4_nt1_g1024", "blocks_wg1024_g256_r2_x0"):
        print(f"  {k:32s} {v['GB/s_median']:8.1f}")
PY
exit $rc
