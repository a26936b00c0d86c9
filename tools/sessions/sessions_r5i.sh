#!/bin/bash
# Round 5, session i: the residual pinned at the pass end (RES 1 spills of
# the 20 x 16 / 12 x 16 resident builds), checked runs on the 4-GPU blocks;
# per-pass 20 x 16 tiles on large plates (A/B against the split pipelines);
# counters of the 20 x 16 resident launch on 2048 x 8192; the issue-rate
# probe with packed f32 variants.
B="python bench.py --steps 20 --warmup 5"
R=$PWD
steps=(
 "tests|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_tile.py tests/test_gpu_converge_gated.py"
 "c20_2048x8192|120|$B --nx 2048 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "c50_2048x8192|120|$B --nx 2048 --ny 8192 --init ref-wrap --converge --check-interval 50"
 "c20_1024|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "c50_1024|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 50"
 "b2048x8192|120|$B --nx 2048 --ny 8192"
 "b1024|120|$B --nx 1024 --ny 8192"
 "b1024_noresident|120|HEAT_TB_RESIDENT=0 $B --nx 1024 --ny 8192"
 "bench|120|$B"
 "t8192_20x16|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_MAX=100000 HEAT_TB_TILE_ROWS=20 HEAT_TB_TILE_WAVES=16 $B"
 "t8192_plan|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_MAX=100000 $B"
 "t2048x8192_20x16|120|HEAT_TB_TRACE=1 HEAT_TB_RESIDENT=0 HEAT_TB_TILE_MAX=100000 HEAT_TB_TILE_ROWS=20 HEAT_TB_TILE_WAVES=16 $B --nx 2048 --ny 8192"
 "t4096x8192_20x16|120|HEAT_TB_TRACE=1 HEAT_TB_TILE_MAX=100000 HEAT_TB_TILE_ROWS=20 HEAT_TB_TILE_WAVES=16 $B --nx 4096 --ny 8192"
 "b4096x8192|120|$B --nx 4096 --ny 8192"
 "bench_2|120|$B"
 "b2048x4096|120|$B --nx 2048 --ny 4096"
 "b1024_2|120|$B --nx 1024 --ny 8192"
 "probe|120|build/probes/stencil_chain"
 "pmc2048|600|PROG=bench.py ARGS='--nx 2048 --ny 8192 --steps 2 --warmup 1 --no-verify' OUT=r5i/pmc2048 bash tools/prof_counters.sh && python3 tools/prof_summary.py --pmc gpurun_out/r5i/pmc2048 --match tile_resident --out gpurun_out/r5i/pmc2048.md"
)
exec bash tools/gpu_run.sh r5i "${steps[@]}"
