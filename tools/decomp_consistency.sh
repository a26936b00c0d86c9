#!/bin/bash
# Bitwise decomposition invariance at full size with the default planner
# (auto depth, split pipelines, m = 8 deep halos): 1, 2, 4 and 8 loopback
# ranks on one GPU must produce the same checksum of the 8192^2 plate.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for g in 1 2 4 8; do
  timeout -k 5 120 ./build/heat --gpus $g --nx 8192 --ny 8192 --steps 1000 --init random --seed 5 \
      --decomp rows --out gpurun_out/ck_$g.txt --out-format checksum --json > gpurun_out/ck_$g.json 2>&1 || exit 1
  echo "gpus=$g $(cat gpurun_out/ck_$g.txt | head -3 | tr '\n' ' ') $(grep -o '"tb_depth": [0-9]*' gpurun_out/ck_$g.json)"
done
