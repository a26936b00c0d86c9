#!/bin/bash
# Round 5, session j: resident tile shapes on the 8-GPU per-rank plates (two
# workgroups per CU vs one 16-wave tile), and where a resident pass's time
# goes (HEAT_TB_RES_DIAG timing builds: 1 no neighbour wait, 3 + no ghost
# reload, 7 + no publish -- wrong results, timing only); the packed f32
# tile update (HEAT_TILE_PK=1 build in build/pk, HEAT_LIB) against the
# scalar one, interleaved.
B="python bench.py --steps 20 --warmup 5"
PK="HEAT_LIB=build/pk/lib/libheat.so"
steps=(
 "b1024|120|$B --nx 1024 --ny 8192"
 "b1024_14x8|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_ROWS=14 HEAT_TB_TILE_WAVES=8 $B --nx 1024 --ny 8192"
 "b1024_13x8|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_ROWS=13 HEAT_TB_TILE_WAVES=8 $B --nx 1024 --ny 8192"
 "b1024_16x8|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_ROWS=16 HEAT_TB_TILE_WAVES=8 $B --nx 1024 --ny 8192"
 "b2048x4096|120|$B --nx 2048 --ny 4096"
 "b2048x4096_14x8|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_ROWS=14 HEAT_TB_TILE_WAVES=8 $B --nx 2048 --ny 4096"
 "b2048x4096_16x8|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_ROWS=16 HEAT_TB_TILE_WAVES=8 $B --nx 2048 --ny 4096"
 "b1192|120|$B --nx 1192 --ny 8192"
 "d1_1024|120|HEAT_TB_RES_DIAG=1 $B --nx 1024 --ny 8192 --no-verify"
 "d3_1024|120|HEAT_TB_RES_DIAG=3 $B --nx 1024 --ny 8192 --no-verify"
 "d7_1024|120|HEAT_TB_RES_DIAG=7 $B --nx 1024 --ny 8192 --no-verify"
 "d7_2048x8192|120|HEAT_TB_RES_DIAG=7 $B --nx 2048 --ny 8192 --no-verify"
 "b1024_2|120|$B --nx 1024 --ny 8192"
 "b1024_14x8_2|120|HEAT_TB_TILE_ROWS=14 HEAT_TB_TILE_WAVES=8 $B --nx 1024 --ny 8192"
 "pk_b1024|120|$PK $B --nx 1024 --ny 8192"
 "b1024|120|$B --nx 1024 --ny 8192"
 "pk_b2048x8192|120|$PK $B --nx 2048 --ny 8192"
 "b2048x8192|120|$B --nx 2048 --ny 8192"
 "pk_b2048x4096|120|$PK $B --nx 2048 --ny 4096"
 "b2048x4096|120|$B --nx 2048 --ny 4096"
 "pk_c20_1024|120|$PK $B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "c20_1024|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "pk_b1024|120|$PK $B --nx 1024 --ny 8192"
 "b1024|120|$B --nx 1024 --ny 8192"
 "pk_b2048x8192|120|$PK $B --nx 2048 --ny 8192"
 "b2048x8192|120|$B --nx 2048 --ny 8192"
 "pk_tests|600|$PK python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_tile.py"
)
exec bash tools/gpu_run.sh r5j "${steps[@]}"
