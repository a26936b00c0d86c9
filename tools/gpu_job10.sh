#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for I in "" "--interior"; do
timeout -k 10 300 python tools/tb_sweep.py --n 8192 --depths 8 --variants 3,7 --waves=-1,-2 $I > gpurun_out/sweep_int.log 2>&1 || exit 1
echo "mode '$I'"; head -3 gpurun_out/sweep_int.log | cut -c1-140
timeout -k 10 300 python tools/tb_sweep.py --nx 1024 --n 8192 --depths 8 --variants 3,7 --waves=-1 $I > gpurun_out/sweep_int2.log 2>&1 || exit 1
head -2 gpurun_out/sweep_int2.log | cut -c1-140
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 && grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/bench.log
