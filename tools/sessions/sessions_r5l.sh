#!/bin/bash
# Round 5, session l: what the split kernel's output stores cost.
# A/B on the 8192^2 bench, interleaved: default build, non-temporal stores
# (HEAT_TB_NTSTORE=1 build of tb_split.o), and the diagnostics build whose
# stores all hit one row per unit (HEAT_TB_DIAG_FIXEDSTORE=1: the same store
# instructions without the HBM write stream; wrong results, --no-verify).
B="python bench.py --steps 20 --warmup 5"
NT="HEAT_LIB=build/exp_nt/libheat.so"
FX="HEAT_LIB=build/exp_fx/libheat.so"
steps=(
 "bench|120|$B"
 "nt|120|$NT $B"
 "fx|120|$FX $B --no-verify"
 "bench|120|$B"
 "nt|120|$NT $B"
 "fx|120|$FX $B --no-verify"
 "bench|120|$B"
 "nt|120|$NT $B"
 "fx|120|$FX $B --no-verify"
)
exec bash tools/gpu_run.sh r5l "${steps[@]}"
