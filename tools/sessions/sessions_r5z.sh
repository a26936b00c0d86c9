#!/bin/bash
# Round 5, session z: chained passes with the streaming build's
# non-temporal stores (not write-through) -- with and without the waits
# (both timing only: cross-XCD visibility needs the sc1 stores), against the
# sc1 chain and one launch per pass, 8192^2.
B="python bench.py --steps 20 --warmup 5 --no-verify"
L() { echo "HEAT_LIB=build/exp_$1/libheat.so"; }
steps=()
for r in 1 2; do
  steps+=("chain|120|$B" "ntnw|120|$(L cntnw) $B" "nt|120|$(L cnt) $B" "nochain|120|HEAT_TB_CHAIN=0 $B")
done
exec bash tools/gpu_run.sh r5z "${steps[@]}"
