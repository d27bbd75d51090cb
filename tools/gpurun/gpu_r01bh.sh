#!/bin/bash
# per-call latency of one SST-file batch (generic path launch overheads)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/percall.py > gpurun_out/bh_percall.json 2> gpurun_out/bh_percall.err
rc=$?
cat gpurun_out/bh_percall.json; tail -2 gpurun_out/bh_percall.err
exit $rc
