#!/bin/bash
# Round 5, session ag: inner-level residual units with plain rows (default)
# against streaming rows (build exp_rlnt, HEAT_LIB), checked runs every 20
# steps on the 2-GPU plate and at 8192^2, interleaved.
B="python bench.py --steps 20 --warmup 5 --init ref-wrap --converge --check-interval 20"
NT="HEAT_LIB=build/exp_rlnt/libheat.so"
steps=()
for r in 1 2; do
  steps+=("p2|120|$B --nx 4096 --ny 8192" "nt_p2|120|$NT $B --nx 4096 --ny 8192"
          "c20|120|$B" "nt_c20|120|$NT $B")
done
exec bash tools/gpu_run.sh r5ag "${steps[@]}"
