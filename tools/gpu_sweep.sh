#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/pytest_kernels.log 2>&1 || { tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -2 gpurun_out/pytest_kernels.log
timeout -k 10 400 python tools/tb_sweep.py --depths ${DEPTHS:-4,6,8} --variants ${VARIANTS:-0,1,2,3} --waves=${WAVES:--1,-2,-3,-4} --json gpurun_out/sweep.json 2>&1 | tee gpurun_out/sweep.log
