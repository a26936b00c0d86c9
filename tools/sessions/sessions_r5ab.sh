#!/bin/bash
# Round 5, session ab: the chained kernel's parallel flag reset (bitwise
# tests), the kernel tests, and the default bench after the rebuild.
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
steps=(
 "tests|600|$T tests/test_gpu_chain.py tests/test_gpu_kernels.py tests/test_gpu_solver.py"
 "bench|120|python bench.py --steps 20 --warmup 5"
)
exec bash tools/gpu_run.sh r5ab "${steps[@]}"
