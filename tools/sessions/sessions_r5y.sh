#!/bin/bash
# Round 5, session y: where the chained passes lose time.  8192^2 bench:
# chains (sc1 stores, s_sleep 1 polls) vs sc1 nt stores (aux 18), s_sleep 8
# polls, no waits at all (diagnostics: wrong results) and one launch per pass.
B="python bench.py --steps 20 --warmup 5"
L() { echo "HEAT_LIB=build/exp_c$1/libheat.so"; }
steps=()
for r in 1 2; do
  steps+=("chain|120|$B" "aux18|120|$(L aux18) $B" "sl8|120|$(L sl8) $B"
          "nowait|120|$(L nowait) $B --no-verify" "nochain|120|HEAT_TB_CHAIN=0 $B")
done
exec bash tools/gpu_run.sh r5y "${steps[@]}"
