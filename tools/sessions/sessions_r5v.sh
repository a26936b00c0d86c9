#!/bin/bash
# Round 5, session v: depth-8 split default on whole-GPU plates (tests +
# bench) and per-wave timelines of one streaming depth-12 pass (8192^2) and
# of the plain one (4096 x 8192): how much of a launch is its tail.
B="python bench.py --steps 20 --warmup 5"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
steps=(
 "tests|600|$T tests/test_gpu_kernels.py tests/test_gpu_converge_gated.py tests/test_gpu_solver.py"
 "bench|120|$B"
 "bench|120|$B"
 "tl8192|120|python tools/wave_timeline.py --nx 8192 --ny 8192 --depth 12"
 "tl4096|120|python tools/wave_timeline.py --nx 4096 --ny 8192 --depth 12"
 "tl8192_d8|120|python tools/wave_timeline.py --nx 8192 --ny 8192 --depth 8"
)
exec bash tools/gpu_run.sh r5v "${steps[@]}"
