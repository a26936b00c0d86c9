#!/bin/bash
# 131072^2 on one GPU, the current library vs the one before the per-
# workgroup residual atomics (abprev/libheat.so, commit 61eda54), interleaved
# on one box: no check and check every 50, 1000 iterations each.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3c5ab
mkdir -p $O
( while sleep 30; do date > $O/heartbeat; done ) &
HB=$!
for rep in 1 2; do
for lib in new old; do
  L=""; [ $lib = old ] && L="$PWD/abprev/libheat.so"
  for c in none 50; do
    if [ $c = none ]; then X=""; else X="--converge --check-interval 50"; fi
    HEAT_LIB=$L timeout -k 10 400 python bench.py --nx 131072 --ny 131072 --steps 1 --warmup 1 --iters-per-step 1000 --init ref-wrap --no-verify $X > $O/big_${lib}_${c}_$rep.log 2>&1 || { kill $HB; tail -20 $O/big_${lib}_${c}_$rep.log; exit 1; }
    echo "$rep $lib $c $(tail -1 $O/big_${lib}_${c}_$rep.log | cut -c80-125)"
  done
done
done
kill $HB
echo done
