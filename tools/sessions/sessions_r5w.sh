#!/bin/bash
# Round 5, session w: chained level-split passes (tb_chain.hip) -- bitwise
# tests against one launch per pass, then the 8192^2 bench with chains
# (default) against HEAT_TB_CHAIN=0, interleaved.
B="python bench.py --steps 20 --warmup 5"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
steps=(
 "chain_tests|600|$T tests/test_gpu_chain.py"
 "bench|120|$B"
 "nochain|120|HEAT_TB_CHAIN=0 $B"
 "bench|120|$B"
 "nochain|120|HEAT_TB_CHAIN=0 $B"
 "bench|120|$B"
 "nochain|120|HEAT_TB_CHAIN=0 $B"
)
exec bash tools/gpu_run.sh r5w "${steps[@]}"
