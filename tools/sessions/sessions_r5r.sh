#!/bin/bash
# Round 5, session r: per-pass workgroup tiles (kTile, forced) on the plates
# the level-split pipelines run: 4096 x 8192 (2-GPU ranks) and 8192^2.
B="python bench.py --steps 20 --warmup 5"
T="HEAT_TB_VARIANT=131088"
steps=()
for s in "--nx 4096 --ny 8192" ""; do
  n=$( [ -z "$s" ] && echo 8192 || echo p2 )
  steps+=("split_$n|120|$B $s"
          "t20x16_$n|120|$T HEAT_TB_TILE_ROWS=20 HEAT_TB_TILE_WAVES=16 $B $s"
          "t12x16_$n|120|$T HEAT_TB_TILE_ROWS=12 HEAT_TB_TILE_WAVES=16 $B $s"
          "t32x8_$n|120|$T HEAT_TB_TILE_ROWS=32 HEAT_TB_TILE_WAVES=8 $B $s")
done
exec bash tools/gpu_run.sh r5r "${steps[@]}"
