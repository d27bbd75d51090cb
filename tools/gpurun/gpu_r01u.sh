#!/bin/bash
# xor3 (v_bitop3) + and_or realign addressing: parity, A/B vs the previous commit, power/clock
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/u_tests.log 2>&1 && \
timeout -k 10 500 python tools/variants.py run --only head base nofold --gib 64 --reps 7 > gpurun_out/u_variants.json 2>gpurun_out/u_variants.err && \
timeout -k 10 200 python tools/power_probe.py --only head base --seconds 5 > gpurun_out/u_power.log 2>&1
rc=$?
tail -3 gpurun_out/u_tests.log
python - <<'PY'
import json
try:
    d = json.load(open("gpurun_out/u_variants.json"))
    print(d["agree"])
    for w, r in d["results"].items():
        print(w, {n: v["GB/s_median"] for n, v in r.items()})
except Exception as e:
    print("variants:", e)
for n in ["head", "base"]:
    try:
        rows = [json.loads(l) for l in open(f"gpurun_out/power_{n}.txt")]
        v = []
        for r in rows:
            try:
                d = json.loads(r["out"])["card0"]
                v.append((d["Current Socket Graphics Package Power (W)"], d["sclk clock speed:"]))
            except Exception:
                pass
        print(n, v[2:6])
    except Exception as e:
        print(n, e)
PY
tail -2 gpurun_out/u_power.log
exit $rc
