#!/bin/bash
# TB depth sweep over the per-rank slab heights of 8192^2 (rows
# decomposition on 8/4/2/1 GPUs), default variant, planner's wave count.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/sweep_depth.jsonl
DEPTHS=${DEPTHS:-4,6,8,10,12,16}
: > $OUT
for nx in 1024 2048 4096 8192; do
  if [[ $nx == 8192 ]]; then plate=""; else plate="--plate-nx 8192 --gx0 $(( (8192 - nx) / 2 ))"; fi
  timeout -k 10 240 python tools/tb_sweep.py --nx $nx --n 8192 $plate --depths $DEPTHS --variants 23 \
      --waves 0 --iters 480 --rounds 5 >> $OUT 2>gpurun_out/sweep_depth.err || exit 1
done
cat $OUT
