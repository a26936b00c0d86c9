#!/bin/bash
# Round 5, session u: the two depth-8 remainder passes of 1000 = 82 x 12 +
# 8 + 8 as level-split pipelines (HEAT_TB_VARIANT=2071 forces the split
# build at every depth; the default runs depth 8 single-wave) at 8192^2.
B="python bench.py --steps 20 --warmup 5"
steps=()
for r in 1 2 3; do
  steps+=("bench|120|$B" "split8|120|HEAT_TB_VARIANT=2071 $B")
done
exec bash tools/gpu_run.sh r5u "${steps[@]}"
