#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for I in "" "--interior"; do
timeout -k 10 300 python tools/tb_sweep.py --n 8192 --depths 8 --variants 0,2,3,4,6,7 --waves=-1,-2 $I > gpurun_out/s1.log 2>&1 || exit 1
echo "8192 mode '$I'"; head -5 gpurun_out/s1.log | cut -c1-125
timeout -k 10 300 python tools/tb_sweep.py --nx 1024 --n 8192 --depths 8 --variants 0,2,3,4,6,7 --waves=-1,-2 $I > gpurun_out/s2.log 2>&1 || exit 1
echo "1024 mode '$I'"; head -4 gpurun_out/s2.log | cut -c1-125
done
