#!/bin/bash
# Round 5, session m: cache policy of the split kernel's row traffic.
# Default build = non-temporal output stores (HEAT_TB_NTSTORE 1); base = the
# previous build (plain stores); ntld = + non-temporal input loads; buf2 /
# buf19 = buffer stores with cache-policy bits nt / sc0 sc1 nt.  8192^2
# interleaved, then the 2-GPU plate (4096 x 8192: 134 MB, inside the MALL)
# and the 131072^2 plate, base against default.
B="python bench.py --steps 20 --warmup 5"
L() { echo "HEAT_LIB=build/exp_$1/libheat.so"; }
steps=()
for r in 1 2; do
  steps+=("bench|120|$B" "base|120|$(L base) $B" "ntld|120|$(L ntld) $B" "buf2|120|$(L buf2) $B" "buf19|120|$(L buf19) $B")
done
for r in 1 2; do
  steps+=("p2|120|$B --nx 4096 --ny 8192" "base_p2|120|$(L base) $B --nx 4096 --ny 8192")
done
steps+=("big|300|python bench.py --steps 3 --warmup 1 --nx 131072 --ny 131072 --no-verify"
        "base_big|300|$(L base) python bench.py --steps 3 --warmup 1 --nx 131072 --ny 131072 --no-verify")
exec bash tools/gpu_run.sh r5m "${steps[@]}"
