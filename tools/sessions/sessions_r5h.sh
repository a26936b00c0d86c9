#!/bin/bash
# Round 5, session h: 20 x 16 resident tiles for the 4-GPU per-rank blocks
# (2048 x 8192, 4096 x 4096), branch-free last-step stores in the tile and
# resident kernels (no per-row basic blocks: spills gone from the tile RES 1
# builds and the 20 x 16 shape).
B="python bench.py --steps 20 --warmup 5"
steps=(
 "tests|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_tile.py tests/test_gpu_converge_gated.py"
 "b2048x8192|120|HEAT_TB_TRACE=1 $B --nx 2048 --ny 8192"
 "b4096|120|HEAT_TB_TRACE=1 $B --nx 4096 --ny 4096"
 "b2048x8192_split|120|HEAT_TB_RESIDENT=0 $B --nx 2048 --ny 8192"
 "b4096_split|120|HEAT_TB_RESIDENT=0 $B --nx 4096 --ny 4096"
 "b1024|120|HEAT_TB_TRACE=1 $B --nx 1024 --ny 8192"
 "b2048x4096|120|$B --nx 2048 --ny 4096"
 "b1192|120|$B --nx 1192 --ny 8192"
 "c20_2048x8192|120|$B --nx 2048 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "c50_2048x8192|120|$B --nx 2048 --ny 8192 --init ref-wrap --converge --check-interval 50"
 "c20_1024|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "bench|120|$B"
 "b2048x8192_2|120|$B --nx 2048 --ny 8192"
 "b4096_2|120|$B --nx 4096 --ny 4096"
 "prof2048|180|rocprofv3 --kernel-trace --stats -d gpurun_out/r5h/prof2048 -o p -- python3 bench.py --steps 5 --warmup 2 --nx 2048 --ny 8192 --no-verify"
)
exec bash tools/gpu_run.sh r5h "${steps[@]}"
