#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for I in "" "--interior"; do
timeout -k 10 300 python tools/tb_sweep.py --n 8192 --depths 8 --variants 3,7 --waves=-1,-2 $I > gpurun_out/sweep_int.log 2>&1 || exit 1
echo "mode '$I'"; head -4 gpurun_out/sweep_int.log | cut -c1-140
timeout -k 10 300 python tools/tb_sweep.py --nx 1024 --n 8192 --depths 8 --variants 3,7 --waves=-1 $I > gpurun_out/sweep_int2.log 2>&1 || exit 1
head -2 gpurun_out/sweep_int2.log | cut -c1-140
done
