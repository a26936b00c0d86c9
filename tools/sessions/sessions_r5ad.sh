#!/bin/bash
# Round 5, session ad: the level-split age-group weights (older : younger
# blocks' row shares, default 1.7 : 1, tuned in round 2) with the streaming
# rows, 8192^2, interleaved twice.
B="python bench.py --steps 20 --warmup 5"
steps=()
for r in 1 2; do
  for w in "" "1.5,1" "1.9,1" "2.1,1"; do
    n=$( [ -z "$w" ] && echo def || echo w${w/,/_} )
    steps+=("$n|120|HEAT_TB_AGE_WEIGHTS=$w $B")
  done
done
exec bash tools/gpu_run.sh r5ad "${steps[@]}"
