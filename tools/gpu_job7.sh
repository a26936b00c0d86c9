#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/pytest_kernels.log 2>&1 || { tail -30 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
timeout -k 10 300 python tools/tb_sweep.py --n 8192 --depths 6,8 --variants 0,3,4,7 --waves=-1,-2 --json gpurun_out/sweep_ramp_8192.json > gpurun_out/sweep_ramp_8192.log 2>&1 || exit 1
head -5 gpurun_out/sweep_ramp_8192.log | cut -c1-140
for ML in 8 16; do
HEAT_TB_MINLEN=$ML timeout -k 10 300 python tools/tb_sweep.py --nx 1024 --n 8192 --depths 4,6,8 --variants 0,3,4,7 --waves=-1,-2 --iters 400 --json gpurun_out/sweep_ramp_1024_ml$ML.json > gpurun_out/sweep_ramp_1024_ml$ML.log 2>&1 || exit 1
echo "ML $ML"; head -5 gpurun_out/sweep_ramp_1024_ml$ML.log | cut -c1-140
done
