#!/bin/bash
# Round 5, session q: what the masked plate-edge waves of the resident
# tiles cost.  HEAT_TB_RES_DIAG=16 computes the plate's top / bottom rows as
# interior rows (wrong results: timing only), interleaved with the default
# on the 8-GPU (1024 x 8192, 2048 x 4096) and 4-GPU (2048 x 8192) plates.
B="python bench.py --steps 20 --warmup 5"
steps=()
for r in 1 2; do
  for s in "--nx 1024 --ny 8192" "--nx 2048 --ny 4096" "--nx 2048 --ny 8192"; do
    n=$(echo $s | tr -d ' -' | sed 's/nx/b/;s/ny/x/')
    steps+=("$n|120|$B $s" "e16_$n|120|HEAT_TB_RES_DIAG=16 $B $s --no-verify")
  done
done
exec bash tools/gpu_run.sh r5q "${steps[@]}"
