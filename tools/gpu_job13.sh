#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 ./build/heat --backend hip --nx 8192 --ny 8192 --steps 1000 --out none --json > gpurun_out/cli_gpu.log 2>&1 || { cat gpurun_out/cli_gpu.log; exit 1; }
tail -1 gpurun_out/cli_gpu.log
timeout -k 10 120 ./build/heat --backend hip --nx 20 --ny 20 --steps 10000 --converge --naming cuda --json > gpurun_out/cli_cuda.log 2>&1 || { cat gpurun_out/cli_cuda.log; exit 1; }
head -2 gpurun_out/cli_cuda.log; ls out_cuda_* 
timeout -k 10 900 python bench/run_configs.py --configs 2,5 --capacity-1gpu > gpurun_out/configs.log 2>&1 || { tail -30 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log
cp bench/results/*.json gpurun_out/ 2>/dev/null
