#!/bin/bash
# Round 5, session aa: pipelines per launch on the 2-GPU plate (4096 x
# 8192: 73-row chunks at the default 2048 units) and at 8192^2.
B="python bench.py --steps 20 --warmup 5"
steps=()
for r in 1 2; do
  for w in 0 1536 1024 2560; do
    steps+=("p2_w$w|120|HEAT_TB_WAVES=$w $B --nx 4096 --ny 8192")
  done
done
for w in 0 1536; do steps+=("b_w$w|120|HEAT_TB_WAVES=$w $B"); done
exec bash tools/gpu_run.sh r5aa "${steps[@]}"
