#!/bin/bash
# BASELINE config 5 on ONE GPU (131072^2, convergence all-reduce every 50,
# 1000 timed iterations) with the final round-3 build.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r3c5
( while sleep 30; do date > gpurun_out/r3c5/heartbeat; done ) &
HB=$!
timeout -k 10 900 python bench/run_configs.py --configs 5 --capacity-1gpu --out gpurun_out/r3c5 > gpurun_out/r3c5/run.log 2>&1
rc=$?
kill $HB
tail -2 gpurun_out/r3c5/run.log | cut -c1-600
exit $rc
