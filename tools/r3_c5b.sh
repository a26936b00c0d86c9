#!/bin/bash
# 131072^2 on one GPU: no check vs check every 50 (same box), 1000 iterations.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3c5b
mkdir -p $O
( while sleep 30; do date > $O/heartbeat; done ) &
HB=$!
for c in none 50; do
  if [ $c = none ]; then X=""; else X="--converge --check-interval 50"; fi
  timeout -k 10 400 python bench.py --nx 131072 --ny 131072 --steps 1 --warmup 1 --iters-per-step 1000 --init ref-wrap --no-verify $X > $O/big_$c.log 2>&1 || { kill $HB; tail -20 $O/big_$c.log; exit 1; }
  echo "$c $(tail -1 $O/big_$c.log | cut -c80-140)"
done
kill $HB
echo done
