#!/bin/bash
# Quick GPU check after a kernel change: TB kernel + solver tests, a depth
# sweep over the per-rank slab shapes (DEPTHS, default 8,12) and the bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
DEPTHS=${DEPTHS:-8,12} bash tools/sweep_depth.sh || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
