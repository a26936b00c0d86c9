#!/bin/bash
# Round 5, session e: what the RES 1 resident build costs by itself
# (HEAT_TB_RES_DIAG_RES1: residual instantiation without checks).
B="python bench.py --steps 20 --warmup 5 --nx 1024 --ny 8192 --init ref-wrap"
steps=(
 "u|120|$B"
 "u_res1|120|HEAT_TB_RES_DIAG_RES1=1 $B"
 "c20|120|$B --converge --check-interval 20"
 "c50|120|$B --converge --check-interval 50"
 "c100|120|$B --converge --check-interval 100"
 "u2|120|$B"
 "u_res1b|120|HEAT_TB_RES_DIAG_RES1=1 $B"
 "c20b|120|$B --converge --check-interval 20"
)
exec bash tools/gpu_run.sh r5e "${steps[@]}"
