#!/bin/bash
# Whole-run A/B of the multi-rank depth choice on ONE GPU: heat --gpus N
# (loopback ranks as threads sharing the device) at 8192^2, default (auto
# depth/variant) vs HEAT_TB_DEPTH=8, rows and 2-D layouts.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/depth_ab.jsonl; : > $out
for n in 4 8; do
  for d in rows 2d; do
    for depth in auto 8; do
      env_depth=""; [ $depth = 8 ] && env_depth="HEAT_TB_DEPTH=8"
      line=$(env $env_depth timeout -k 10 120 build/heat --gpus $n --nx 8192 --ny 8192 --steps 2000 --decomp $d --init random --out none --json 2>/dev/null | tail -1) || exit 1
      echo "{\"n\": $n, \"decomp\": \"$d\", \"depth\": \"$depth\", \"run\": $line}" | tee -a $out | cut -c1-160
    done
  done
done
