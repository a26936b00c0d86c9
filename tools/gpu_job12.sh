#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run() { timeout -k 10 300 python tools/tb_sweep.py --depths ${D:-8} --variants ${V:-0,3,4,7} --waves=-1 "$@" > gpurun_out/s.log 2>&1 || exit 1; echo "== $*"; head -2 gpurun_out/s.log | cut -c1-118; }
run --n 8192
run --n 8192 --interior
run --nx 1024 --n 8192
run --nx 1024 --n 8192 --plate-nx 8192 --gx0 4096
D=4,6,8 run --nx 1024 --n 8192 --plate-nx 8192 --gx0 0
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 && grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/bench.log
