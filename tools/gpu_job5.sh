#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for NX in 1024 2048; do
  timeout -k 10 300 python tools/tb_sweep.py --nx $NX --n 8192 --depths 2,4,6,8 --variants 0,4 --waves=-1,-2,-3 --iters 400 --json gpurun_out/sweep_nx$NX.json > gpurun_out/sweep_nx$NX.log 2>&1 || exit 1
  head -8 gpurun_out/sweep_nx$NX.log | cut -c1-170
done
