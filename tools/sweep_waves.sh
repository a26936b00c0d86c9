#!/bin/bash
# Waves-per-SIMD sweep of the TB kernel over slab heights (the per-rank
# shapes of 8192^2 on 1/2/4/8 GPUs, rows decomposition).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/sweep_waves.jsonl
: > $OUT
for nx in 512 1024 2048 4096 8192; do
  if [[ $nx == 8192 ]]; then plate=""; else plate="--plate-nx 8192 --gx0 $(( (8192 - nx) / 2 ))"; fi
  timeout -k 10 200 python tools/tb_sweep.py --nx $nx --n 8192 $plate --depths 8 --variants 7 \
      --waves 0,1024,2048,3072 --iters 400 --rounds 5 >> $OUT 2>/dev/null || exit 1
done
cat $OUT
