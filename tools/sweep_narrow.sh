#!/bin/bash
# float4 (variant 23) vs float2-lane (variant 87) TB strips over slab heights
# and waves targets.  Output: gpurun_out/sweep_narrow.jsonl
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/sweep_narrow.jsonl
: > $OUT
for nx in 1024 2048 4096 8192; do
  if [[ $nx == 8192 ]]; then plate=""; else plate="--plate-nx 8192 --gx0 $(( (8192 - nx) / 2 ))"; fi
  timeout -k 10 240 python tools/tb_sweep.py --nx $nx --n 8192 $plate --depths 8 --variants 23,87 \
      --waves 0,1024,2048,3072,4096,5120 --iters 400 --rounds 5 >> $OUT 2>/dev/null || exit 1
done
cat $OUT
