#!/bin/bash
# Round 5, session n: the streaming level-split build (tb_split_nt.hip)
# chosen by the bytes a pass sweeps: GPU tests, 8192^2 / 2-GPU-plate /
# checked benches with the planner trace (nt 1 / nt 0 in the "[heat tb]"
# lines).
B="python bench.py --steps 20 --warmup 5"
steps=(
 "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
 "bench|120|HEAT_TB_TRACE=1 $B"
 "p2|120|HEAT_TB_TRACE=1 $B --nx 4096 --ny 8192"
 "c20_8192|120|$B --init ref-wrap --converge --check-interval 20"
 "bench|120|$B"
 "nt0|120|HEAT_TB_NT=0 $B"
 "bench|120|$B"
 "nt0|120|HEAT_TB_NT=0 $B"
)
exec bash tools/gpu_run.sh r5n "${steps[@]}"
