#!/bin/bash
# Round-2 refresh: GPU suite, smoke, default bench, strong-scaling flag at N=1, secondary workloads
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > $O/r02x_tests.log 2>&1 || exit $?
tail -1 $O/r02x_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r02x_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/r02x_bench.json 2> $O/r02x_bench.err || exit $?
cat $O/r02x_bench.json
timeout -k 10 300 python bench.py --strong --no-gather --steps 5 --warmup 1 --no-cpu-baseline > $O/r02x_bench_strong.json 2>&1 || exit $?
cat $O/r02x_bench_strong.json
timeout -k 10 900 python tools/bench_configs.py --reps 5 > $O/r02x_configs.json 2> $O/r02x_configs.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r02x_configs.json"))
for k, v in d["results"].items():
    print(k, v["GiB/s"], v["roofline_frac"])
PY
