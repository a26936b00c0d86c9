#!/bin/bash
# Round 5, session k: packed f32 row update on 12-row tile waves (RES 0),
# bitwise tests; A/B of buffer stores in the streaming / level-split
# kernels' main loops (HEAT_TB_BUFSTORE=1 build in build/st, HEAT_LIB)
# against the global stores, interleaved on the 8192^2 bench.
B="python bench.py --steps 20 --warmup 5"
ST="HEAT_LIB=build/st/lib/libheat.so"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
steps=(
 "tests|900|$T tests/test_gpu_resident.py tests/test_gpu_tile.py tests/test_gpu_converge_gated.py tests/test_gpu_kernels.py"
 "st_tests|900|$ST $T tests/test_gpu_kernels.py tests/test_gpu_converge_gated.py tests/test_gpu_solver.py"
 "bench|120|$B"
 "st_bench|120|$ST $B"
 "bench|120|$B"
 "st_bench|120|$ST $B"
 "bench|120|$B"
 "st_bench|120|$ST $B"
 "b1024|120|$B --nx 1024 --ny 8192"
 "b2048x4096|120|$B --nx 2048 --ny 4096"
 "b2048x8192|120|$B --nx 2048 --ny 8192"
 "c20_1024|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "b1192|120|$B --nx 1192 --ny 8192"
 "c20_8192|120|$B --init ref-wrap --converge --check-interval 20"
 "st_c20_8192|120|$ST $B --init ref-wrap --converge --check-interval 20"
 "b4096x8192|120|$B --nx 4096 --ny 8192"
 "st_b4096x8192|120|$ST $B --nx 4096 --ny 8192"
 "b1024_2|120|$B --nx 1024 --ny 8192"
)
exec bash tools/gpu_run.sh r5k "${steps[@]}"
