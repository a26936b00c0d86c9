#!/bin/bash
# Round 5, session af: inner-level residual passes with streaming rows
# (tb_split_rl{a,b,c}.hip): their tests, then checked 8192^2 runs (every
# 20 / 50, ref-wrap) and the checked 2-GPU plate.
B="python bench.py --steps 20 --warmup 5 --init ref-wrap"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
steps=(
 "tests|600|$T tests/test_gpu_kernels.py tests/test_gpu_converge_gated.py tests/test_gpu_solver.py"
 "c20|120|$B --converge --check-interval 20"
 "c50|120|$B --converge --check-interval 50"
 "ref|120|$B"
 "c20|120|$B --converge --check-interval 20"
 "c50|120|$B --converge --check-interval 50"
 "ref|120|$B"
 "p2_c20|120|$B --converge --check-interval 20 --nx 4096 --ny 8192"
)
exec bash tools/gpu_run.sh r5af "${steps[@]}"
