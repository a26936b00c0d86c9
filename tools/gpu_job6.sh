#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for ML in 8 16 32; do
  HEAT_TB_MINLEN=$ML timeout -k 10 300 python tools/tb_sweep.py --nx 1024 --n 8192 --depths 4,8 --variants 0,1,4,5 --waves=-1,-2,-4 --iters 400 --json gpurun_out/sweep_ml$ML.json > gpurun_out/sweep_ml$ML.log 2>&1 || exit 1
  echo "minlen $ML"; head -4 gpurun_out/sweep_ml$ML.log | cut -c1-150
done
