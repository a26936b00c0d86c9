#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run() { timeout -k 10 300 python tools/tb_sweep.py --depths ${D:-8} --variants ${V:-3,7,11,15} --waves=${W:--1} "$@" > gpurun_out/s.log 2>&1 || exit 1; echo "== $*"; head -4 gpurun_out/s.log | cut -c1-130; }
run --n 8192 --rounds 7
W=-1,-2 run --nx 1024 --n 8192 --plate-nx 8192 --gx0 4096
