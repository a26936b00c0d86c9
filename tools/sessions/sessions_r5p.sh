#!/bin/bash
# Round 5, session p: MALL-sized plates.  4096 x 8192 (plain rows by
# default) against non-temporal loads with plain stores (build
# exp_ldonly, HEAT_LIB); 6144 x 8192 (201 MB, just above kTbStreamBytes:
# streaming by default) against HEAT_TB_NT=0.
B="python bench.py --steps 20 --warmup 5"
LD="HEAT_LIB=build/exp_ldonly/libheat.so"
steps=()
for r in 1 2; do
  steps+=("p2|120|$B --nx 4096 --ny 8192" "ld_p2|120|$LD $B --nx 4096 --ny 8192"
          "p6k|120|$B --nx 6144 --ny 8192" "nt0_p6k|120|HEAT_TB_NT=0 $B --nx 6144 --ny 8192")
done
exec bash tools/gpu_run.sh r5p "${steps[@]}"
